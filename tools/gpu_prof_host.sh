#!/bin/bash
# Host-phase profile (GK_PROFILE=1) of bench.py per config (no aux): one log per config under
# gpurun_out/.  Usage: bash tools/gpu_prof_host.sh TAG [CONFIGS]   (default "C2 C3")
tag=${1:-hp}; cfgs=${2:-C2 C3}
mkdir -p gpurun_out
for c in $cfgs; do
  GK_PROFILE=1 timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-aux --no-cpu-baseline \
      > gpurun_out/${tag}_${c}.log 2>&1 || exit $?
done
exit 0
