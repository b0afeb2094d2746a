set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
args=()
for v in base bw3 bw4 bk4 cs256 cs512; do
  lib=""; [ $v != base ] && lib="PBA_LIBRARY=$PWD/variants/libpba_$v.so"
  args+=(240 gpurun_out/r6_intr_probe20_$v.log env $lib rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/intr6t_$v -o run -- python3 tools/probe/intr_probe.py @@)
done
unset 'args[${#args[@]}-1]'
bash tools/gpu_steps.sh "${args[@]}"
