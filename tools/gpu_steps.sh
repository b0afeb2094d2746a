#!/bin/bash
# Runs GPU steps in order, each under its own time limit; a test failure (exit 1) goes on to the next step, anything
# else (a time limit 124/137, an abort 134, a segfault 139, …) ends the call there.
#   tools/gpu_steps.sh <seconds> <log> <command...> [@@ <seconds> <log> <command...>]...
# (steps are separated by @@, so a command may hold the -- of rocprofv3)
set -u
while [ $# -gt 0 ]; do
  secs=$1; log=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "@@" ]; do cmd+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  timeout -k 10 "$secs" "${cmd[@]}" > "$log" 2>&1
  rc=$?
  echo "step rc=$rc: ${cmd[*]}" >> gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
