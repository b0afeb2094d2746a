set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
 600 gpurun_out/r6_arrow_t29.log python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_distributed.py tests/test_gpu_configs.py -k "arrow or free_intrinsics or front_and_global or optimize_intrinsics or solver_paths or intrinsics or point_sums" @@ \
 240 gpurun_out/r6_intr_plain29.log python3 tools/probe/intr_probe.py @@ \
 240 gpurun_out/r6_intr_probe29.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/intr7a -o run -- python3 tools/probe/intr_probe.py
