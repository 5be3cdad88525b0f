#!/bin/bash
# SQ counter passes (tools/sq_counters2.sh) for the in-tree library and, when given, a variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/sq_counters2.sh || exit $?
python tools/sq_summary.py gpurun_out/sq/run_results.db > gpurun_out/sq_summary.txt 2>&1
python tools/sq_summary.py gpurun_out/sq2/run_results.db > gpurun_out/sq2_summary.txt 2>&1
exit 0
