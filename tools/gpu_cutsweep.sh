#!/bin/bash
# GK_T1ENC_CUTS sweep on C2 and C3 (bench.py, no aux): one log per (value, config).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $SWEEP_VALUES; do
  for c in C2 C3; do
    GK_T1ENC_CUTS=$v timeout -k 10 240 python bench.py --config $c --steps 6 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/var_${c}_$v.log 2>&1 || exit $?
  done
done
exit 0
