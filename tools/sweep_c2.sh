#!/bin/bash
# C2 bench under a list of environment settings (one GPU process each, its own time limit);
# one line per setting with the stage times, into gpurun_out/sweep.txt.
# Usage: bash tools/sweep_c2.sh "ENV1=a ENV2=b" "ENV1=c" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "$@"; do
    env $s timeout -k 10 180 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-aux > gpurun_out/sweep_run.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$s rc=$rc" >> gpurun_out/sweep.txt; tail -5 gpurun_out/sweep_run.log >> gpurun_out/sweep.txt; exit $rc; fi
    python - "$s" >> gpurun_out/sweep.txt <<'EOF'
import json, sys
l = [x for x in open("gpurun_out/sweep_run.log") if x.startswith("{")][-1]
d = json.loads(l)
st = d["stages_ms"]
print("%-40s value %8.1f ms %7.3f enc_t1 %6.3f enc_t2 %6.3f dec_t1 %6.3f dec_t2 %6.3f" % (
    sys.argv[1], d["value"], d["ms_per_step"], st["enc_t1_ms"], st["enc_t2_ms"], st["dec_t1_ms"], st["dec_t2_ms"]))
EOF
done
