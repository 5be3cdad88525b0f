#!/bin/bash
# C3 encode T1 with the heaviest first-chunk blocks on solo MQ waves (GK_T1ENC_SOLO = count), then
# the default bench line.  Each GPU step has its own limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${SOLO_SWEEP:-0 128 512 0}; do
    GK_T1ENC_SOLO=$n timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 2 --no-aux --no-cpu-baseline \
        > gpurun_out/solo_$n.json 2>&1 || exit $?
    python - "$n" <<'PY'
import json, sys
t = open("gpurun_out/solo_%s.json" % sys.argv[1]).read()
d = json.loads(t[t.index("{"):])
m = d["stages_ms"]
print("solo", sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "enc_t1", m["enc_t1_ms"], "cm", m.get("enc_t1_cm_ms"), "coder", m.get("enc_t1_coder_ms"), "enc_t2", m["enc_t2_ms"], "dec_t2", m["dec_t2_ms"], flush=True)
PY
done
timeout -k 10 500 python bench.py > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || exit $?
python -c "
import json; t=open('gpurun_out/r06c_bench.json').read(); d=json.loads(t[t.index('{'):])
print('value', d['value'], d['ms_per_step'], {k: v['value'] for k, v in d.get('per_config', {}).items()}, {k: v['value'] for k, v in d.get('aux', {}).items()})"
