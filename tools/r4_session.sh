#!/bin/bash
# Round-4 GPU session: distributed + GN tests, a short bench at N = 1 (with the 1/8-shard leg), the N = 2 bench path
# rehearsed with gloo on this one GPU, and a kernel trace of one distributed-loop trial.  Each GPU step has its own time
# limit; the script stops at the first crash / timeout (tools/gpu_steps.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  600 gpurun_out/s_tests.log python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_distributed.py tests/test_gpu_gn.py -rf @@ \
  400 gpurun_out/s_bench.log python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --no-c5 @@ \
  300 gpurun_out/s_n2.log env PBA_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --gn-iterations 3 @@ \
  300 gpurun_out/s_dtrace.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s_dtrace -o run -- \
      python tools/probe/dist_trace.py
python tools/gn_trace.py $(ls gpurun_out/s_dtrace/*/run_kernel_trace.csv gpurun_out/s_dtrace/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/s_dtrace.txt 2>&1
cat gpurun_out/steps.txt
