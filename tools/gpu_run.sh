#!/bin/bash
# GPU-box driver for one gpurun call.  Each GPU step has its own time limit;
# a crash / abort / timeout (exit >= 124) stops the script (no further GPU work).
# Usage: bash tools/gpu_run.sh "<steps>"   steps: any of test smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT="$PWD/gpurun_out"
REPO="$PWD"
STEPS="${1:-test smoke bench}"
TESTSEL="${TESTSEL:-tests}"
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*" >> "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >> "$OUT/steps.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> "$OUT/steps.log"; exit $rc; fi
    return 0
}
for s in $STEPS; do
    case $s in
        test) run pytest_gpu 900 python -m pytest $TESTSEL -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
        prof) (cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/prof" -o run -- python "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-aux ${PROF_ARGS:-}) || exit $? ;;
        profaux) (cd /tmp && run profaux 900 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/profaux" -o run -- python "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-}) || exit $? ;;
        pmc) (cd /tmp && run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$REPO/gpurun_out/pmc_fetch" -o run -- python "$REPO/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-aux ${PROF_ARGS:-} && run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$REPO/gpurun_out/pmc_write" -o run -- python "$REPO/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-aux ${PROF_ARGS:-}) || exit $? ;;
    esac
done
exit 0
