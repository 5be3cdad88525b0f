#!/bin/bash
# GPU suite, then bench lines and rocprofv3 kernel statistics per config (no PMC): one gpurun call
# after a kernel change.  Usage: bash tools/gpu_check_perf.sh TAG [CONFIGS]
# Logs: gpurun_out/TAG_pytest_gpu.log, TAG_bench_<cfg>.log, prof_TAG_<cfg>/ (kernel stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-chk}; cfgs=${2:-C2 C3}
OUT=$PWD/gpurun_out; mkdir -p "$OUT"
if [ -z "${SKIP_SUITE:-}" ]; then
  bash tools/gpu_suite.sh "$tag" || exit $?
fi
for c in $cfgs; do
  timeout -k 10 300 python -u bench.py --config $c --steps 8 --warmup 2 --no-aux --no-cpu-baseline \
      > "$OUT/${tag}_bench_$c.log" 2>&1 || exit $?
  tail -1 "$OUT/${tag}_bench_$c.log" | cut -c1-400
done
for c in $cfgs; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${tag}_$c" -o run -- \
      python3 "$OLDPWD/bench.py" --config $c --steps 3 --warmup 1 --no-aux --no-cpu-baseline) \
      > "$OUT/${tag}_prof_$c.log" 2>&1 || exit $?
done
exit 0
