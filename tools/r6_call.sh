set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
args=()
for i in 1 2; do
  for v in prev cur; do
    args+=(240 gpurun_out/r6_ab27_${v}_$i.log env PBA_LIBRARY=$PWD/variants/libpba_$v.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab27_${v}_$i -o run -- python3 tools/probe/intr_probe.py @@)
  done
done
unset 'args[${#args[@]}-1]'
bash tools/gpu_steps.sh "${args[@]}"
