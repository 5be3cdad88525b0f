#!/bin/bash
# One rocprofv3 PMC pass of SQ counters over a 1-step bench (kernel-level issue/stall breakdown).
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d "$GRAFT_REPO_ROOT/gpurun_out/sq" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-aux --no-cpu-baseline ${PROF_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/sq.log" 2>&1
