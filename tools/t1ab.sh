#!/bin/bash
# A/B of the T1 decoder variants / park thresholds on the C2 bench (stats on stderr).
# T1AB="variant:park ..." (default "0:4 1:4 1:8 1:32")
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${T1AB:-0:4 1:4 1:8 1:32}; do
  a=${v%%:*}; b=${v##*:}
  GK_T1DEC=$a GK_T1DEC_PARK=$b GK_T1_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/bench_${a}_${b}.log 2>&1 || exit $?
done
