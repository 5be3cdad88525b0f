#!/bin/bash
# Solo decoder timing (GK_T1_STATS=2): C2 and C3 decoder cycle counts, lane-parallel vs solo waves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GK_T1_STATS=2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-aux --no-cpu-baseline > gpurun_out/timing_c2.log 2>&1 || exit $?
GK_T1_STATS=2 timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 0 --no-aux --no-cpu-baseline > gpurun_out/timing_c3.log 2>&1 || exit $?
