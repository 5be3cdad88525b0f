#!/bin/bash
# C4 host-phase A/B: GK_PROFILE=1 bench.py --config C4 alternating the in-tree library and
# grok_amd/libgrok_amd_old.so on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in 1 2; do
  for v in cur old; do
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    GROK_AMD_LIB=$lib GK_PROFILE=1 timeout -k 10 200 python bench.py --config C4 --steps 4 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/c4ab_${v}_$i.log 2>&1 || exit $?
  done
done
exit 0
