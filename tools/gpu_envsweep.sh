#!/bin/bash
# bench.py (C2, no aux) once per value of environment variable $SWEEP_VAR in $SWEEP_VALUES.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $SWEEP_VALUES; do
    env $SWEEP_VAR=$v timeout -k 10 240 python bench.py --steps 8 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/var_${SWEEP_VAR}_$v.log 2>&1 || exit $?
done
exit 0
