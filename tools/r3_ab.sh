#!/bin/bash
# Round-3 A/B probes on the GPU box (diagnostic): the C5 kernel with / without its camera table, the one-launch PCR
# against a launch per level (pba_solve kernel traces at C4), the distributed loop's trial timeline on one rank and
# the eight-shard rehearsal.  Every step has its own time limit (tools/gpu_steps.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --gn-iterations 0 --steps 100"
tools/gpu_steps.sh \
  200 gpurun_out/c5_ct.txt $B @@ \
  200 gpurun_out/c5_noct.txt env PBA_NO_CAM_TABLE=1 $B @@ \
  200 gpurun_out/c5_ct2.txt $B || exit $?
AB_VAR=PBA_PCR_FUSED GN_ARGS="--solve" timeout -k 10 600 tools/ab_env.sh 0 1 2 > gpurun_out/ab_pcr.txt 2>&1 || exit $?
tools/gpu_steps.sh \
  300 gpurun_out/dist_trace.txt rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dt -o run -- \
      python tools/probe/dist_trace.py @@ \
  400 gpurun_out/rehearsal.txt python tools/probe/rehearsal_probe.py
