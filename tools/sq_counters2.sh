#!/bin/bash
# Two rocprofv3 PMC passes of SQ counters over a 1-step bench: instruction counts and issue/wait
# breakdown per kernel (summarise with tools/sq_summary.py gpurun_out/sq/run_results.db).
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d "$R/gpurun_out/sq" -o run -- python "$R/bench.py" --steps 1 --warmup 0 --no-aux --no-cpu-baseline ${PROF_ARGS:-} > "$R/gpurun_out/sq.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$R/gpurun_out/sq2" -o run -- python "$R/bench.py" --steps 1 --warmup 0 --no-aux --no-cpu-baseline ${PROF_ARGS:-} > "$R/gpurun_out/sq2.log" 2>&1 || exit $?
