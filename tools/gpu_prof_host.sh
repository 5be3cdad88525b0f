#!/bin/bash
# Host-phase profile (GK_PROFILE=1) of bench.py C2 and C3 (no aux): one log per config under
# gpurun_out/.  Usage: bash tools/gpu_prof_host.sh TAG
tag=${1:-hp}
mkdir -p gpurun_out
for c in C2 C3; do
  GK_PROFILE=1 timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-aux --no-cpu-baseline \
      > gpurun_out/${tag}_${c}.log 2>&1 || exit $?
done
grep -h -E "t2|pcrd|decode|value" gpurun_out/${tag}_C2.log | tail -12
