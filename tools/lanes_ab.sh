#!/bin/bash
# A/B of blocks per wave for the T1 decoder / MQ encoder on the C2 bench.
# LANES_AB="declanes:enclanes ..."  (default "64:64 48:48 32:32 24:24 16:16")
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
[ -n "${STATS:-}" ] && export GK_T1_STATS=1
for v in ${LANES_AB:-64:64 48:48 32:32 24:24 16:16}; do
  a=${v%%:*}; b=${v##*:}
  GK_T1DEC_LANES=$a GK_T1ENC_LANES=$b timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-aux --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/lanes_${a}_${b}.log 2>&1 || exit $?
  python - "$a" "$b" <<'PY' >> gpurun_out/lanes_summary.txt
import json, sys
r = json.loads([l for l in open("gpurun_out/lanes_%s_%s.log" % (sys.argv[1], sys.argv[2])) if l.startswith("{")][-1])
s = r["stages_ms"]
print("dec_lanes %s enc_lanes %s value %.1f ms %.2f dec_t1 %.2f enc_t1 %.2f (cm %.2f mq %.2f)" % (
    sys.argv[1], sys.argv[2], r["value"], r["ms_per_step"], s["dec_t1_ms"], s["enc_t1_ms"],
    s.get("enc_t1_cm_ms", 0), s.get("enc_t1_coder_ms", 0)))
PY
done
