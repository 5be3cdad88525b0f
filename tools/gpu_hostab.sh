#!/bin/bash
# Host-phase A/B: GK_PROFILE=1 bench.py (C2 and C3, no aux) alternating the in-tree library and
# grok_amd/libgrok_amd_$ALT.so on one box, so host-side changes compare on the same CPU.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
  for v in cur $ALT; do
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    for c in C2 C3; do
      GROK_AMD_LIB=$lib GK_PROFILE=1 timeout -k 10 200 python bench.py --config $c --steps 4 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/hab_${v}_${c}_$i.log 2>&1 || exit $?
    done
  done
done
exit 0
