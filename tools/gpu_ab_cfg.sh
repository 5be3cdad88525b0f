#!/bin/bash
# A/B of library variants per config: bench.py (no aux) for each "variant:config" pair in $PAIRS
# ("cur" = the in-tree library, else grok_amd/libgrok_amd_<variant>.so).  Logs: gpurun_out/ab_<v>_<c>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pc in $PAIRS; do
    v=${pc%%:*}; c=${pc##*:}
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    GROK_AMD_LIB=$lib timeout -k 10 240 python bench.py --config $c --steps 8 --warmup 2 --no-aux --no-cpu-baseline \
        > gpurun_out/ab_${v}_$c.log 2>&1 || exit $?
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_${v}_$c.log').read().strip().split('\n')[-1]); s=d['stages_ms']
print('$v $c', d['value'], d['ms_per_step'], 'enc_t1', s['enc_t1_ms'], 'dec_t1', s['dec_t1_ms'], 'dec_t1_coder', s.get('dec_t1_coder_ms'))"
done
exit 0
