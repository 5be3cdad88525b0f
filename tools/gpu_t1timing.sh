#!/bin/bash
# T1 decoder cycle split (GK_T1_STATS=2: s_memtime-stamped events vs steps) for the in-tree
# library and the A/B variant grok_amd/libgrok_amd_old.so when present.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
GK_T1_STATS=2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-aux --no-cpu-baseline > gpurun_out/timing_new.log 2>&1 || exit $?
if [ -f grok_amd/libgrok_amd_old.so ]; then
GROK_AMD_LIB=$PWD/grok_amd/libgrok_amd_old.so GK_T1_STATS=2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-aux --no-cpu-baseline > gpurun_out/timing_old.log 2>&1 || exit $?
fi
exit 0
