set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
 600 gpurun_out/r6_arrow_t28.log python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_distributed.py tests/test_gpu_configs.py -k "arrow or free_intrinsics or front_and_global or optimize_intrinsics or solver_paths or intrinsics or point_sums"
