#!/bin/bash
# Decoder launch sweep: critical-lane key (GK_T1DEC_CRIT 1/2/3)
# one short C2 bench each, decoder stats in stderr / the JSON line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 1 2 3; do
    GK_T1DEC_CRIT=$m timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/crit$m.log 2>&1 || exit $?
done
