#!/bin/bash
# Round-6 profile pass: host phase times of C3 (GK_PROFILE), then the kernel trace of the
# headline (C2+C3) bench.  Each GPU step has its own limit; the first failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06}
mkdir -p gpurun_out
REPO="$PWD"
GK_PROFILE=1 timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-aux --no-cpu-baseline \
    > gpurun_out/${TAG}_c3prof.json 2> gpurun_out/${TAG}_c3prof.err || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/${TAG}_prof" -o run -- \
    python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-aux) > "$REPO/gpurun_out/${TAG}_prof.log" 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" > gpurun_out/${TAG}_kernel_stats.txt && head -30 gpurun_out/${TAG}_kernel_stats.txt
