#!/bin/bash
# A/B of the T1 decoder park threshold (GK_T1DEC_PARK) on the C2 bench, with decoder stats.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export GK_T1_STATS=1
for p in ${PARK_AB:-4 8 16}; do
  GK_T1DEC_PARK=$p timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/park_$p.log 2>&1 || exit $?
  python - "$p" <<'PY' >> gpurun_out/park_summary.txt
import json, sys
L = open("gpurun_out/park_%s.log" % sys.argv[1]).read().splitlines()
r = json.loads([l for l in L if l.startswith("{")][-1])
st = [l for l in L if "t1dec stats" in l][-1]
print("park %s value %.1f dec_t1 %.2f | %s" % (sys.argv[1], r["value"], r["stages_ms"]["dec_t1_ms"], st))
PY
done
