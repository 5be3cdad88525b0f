#!/bin/bash
# GPU-box driver: per-config kernel statistics and HBM traffic (one gpurun call).
# For each config in $CONFIGS (default "C2 C3 C4"): rocprofv3 --kernel-trace --stats of a short
# bench run, then two separate PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM
# section: counters in their own runs, no trace domains).  Every GPU step has its own time limit;
# a timeout / crash (exit >= 124) ends the script.
# Usage: bash tools/gpu_profile_all.sh [TAG]    (outputs under gpurun_out/prof_<TAG>_<cfg>*)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPO="$PWD"
OUT="$REPO/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-r04}"
CONFIGS="${CONFIGS:-C2 C3 C4}"
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*" >> "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$t" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >> "$OUT/steps.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> "$OUT/steps.log"; exit $rc; fi
    return $rc
}
for c in $CONFIGS; do
    B="$REPO/bench.py --config $c --no-aux --no-cpu-baseline"
    run "stats_${TAG}_$c" 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_$c" -o run -- python3 $B --steps 3 --warmup 1 || exit $?
    run "pmcf_${TAG}_$c" 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmcf_${TAG}_$c" -o run -- python3 $B --steps 1 --warmup 0 || exit $?
    run "pmcw_${TAG}_$c" 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmcw_${TAG}_$c" -o run -- python3 $B --steps 1 --warmup 0 || exit $?
done
exit 0
