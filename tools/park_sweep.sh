#!/bin/bash
# Decoder event trigger sweep (GK_T1DEC_PARK: parked lanes that start a stripe-boundary event).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for k in 8 16 24; do
  GK_T1DEC_PARK=$k timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/park_$k.log 2>&1 || exit $?
done
