#!/bin/bash
# GPU suite, then one bench line per config (no profiling): the quick check after a change.
# Usage: bash tools/gpu_check_quick.sh TAG [CONFIGS]   (logs: gpurun_out/TAG_*)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-q}; cfgs=${2:-C2 C3 C4}
OUT=$PWD/gpurun_out; mkdir -p "$OUT"
if [ -z "${SKIP_SUITE:-}" ]; then
  bash tools/gpu_suite.sh "$tag" || exit $?
fi
for c in $cfgs; do
  GK_PROFILE=${GK_PROFILE:-} timeout -k 10 300 python -u bench.py --config $c --steps 8 --warmup 2 --no-aux --no-cpu-baseline \
      > "$OUT/${tag}_bench_$c.log" 2>&1 || exit $?
  tail -1 "$OUT/${tag}_bench_$c.log" | cut -c1-200
done
exit 0
