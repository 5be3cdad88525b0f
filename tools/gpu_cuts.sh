#!/bin/bash
# T1 encode chunk cuts (GK_T1ENC_CUTS) per config: bench.py enc_t1 stage for each cut list in $CUTS
# (space-separated, each a comma list).  Logs: gpurun_out/cuts_<i>_<cfg>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in ${CONFIGS:-C2}; do
i=0
for cut in $CUTS; do
    i=$((i+1))
    GK_T1ENC_CUTS=$cut timeout -k 10 240 python bench.py --config $c --steps 6 --warmup 2 --no-aux --no-cpu-baseline \
        > gpurun_out/cuts_${i}_$c.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/cuts_${i}_$c.log').read().strip().split('\n')[-1]); s=d['stages_ms']
print('$c $cut', d['value'], 'enc_t1', s['enc_t1_ms'], 'cm', s.get('enc_t1_cm_ms'), 'coder', s.get('enc_t1_coder_ms'))"
done
done
exit 0
