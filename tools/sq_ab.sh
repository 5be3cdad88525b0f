#!/bin/bash
# SQ counter passes for the two T1 decoder variants (GK_T1DEC=0 / 1).
R="$GRAFT_REPO_ROOT"
cd /tmp
for v in 0 1; do
  GK_T1DEC=$v timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d "$R/gpurun_out/sq$v" -o run -- python "$R/bench.py" --steps 1 --warmup 0 --no-aux --no-cpu-baseline > "$R/gpurun_out/sq$v.log" 2>&1 || exit $?
done
