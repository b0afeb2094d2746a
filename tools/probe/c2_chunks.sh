#!/bin/bash
# Diagnostic: the C2 drop-in probe at a few read-back chunk sizes (PBA_CERES_CHUNK_BLOCKS).
set -u
for c in ${CHUNKS:-4096 16384}; do
  PBA_CERES_CHUNK_BLOCKS=$c timeout -k 10 600 python tools/probe/c2_probe.py > gpurun_out/c2_probe_$c.log 2>&1 || exit $?
done
