#!/bin/bash
# Rehearsal of the bench's N > 1 path on one GPU: N ranks over gloo sharing the device (PBA_BENCH_BACKEND=gloo), N = 2
# and 4; one bench line per N into gpurun_out/rehearse_n<N>.log.  Each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${NS:-2 4}; do
  PBA_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
      > gpurun_out/rehearse_n$n.log 2>&1
  rc=$?
  echo "N=$n rc=$rc"; tail -1 gpurun_out/rehearse_n$n.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
