#!/bin/bash
# bench.py per environment setting: each entry of $RUNS is "NAME:CONFIG:VAR=VAL[,VAR=VAL...]"
# (VAR=VAL may be "-" for none).  Logs: gpurun_out/env_NAME_CONFIG.log; prints a stage line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in $RUNS; do
    name=${r%%:*}; rest=${r#*:}; c=${rest%%:*}; envs=${rest#*:}
    [ "$envs" = "-" ] && envs=""
    env ${envs//,/ } timeout -k 10 240 python bench.py --config $c --steps 8 --warmup 2 --no-aux --no-cpu-baseline \
        > gpurun_out/env_${name}_$c.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/env_${name}_$c.log').read().strip().split('\n')[-1]); s=d['stages_ms']
print('$name $c', d['value'], d['ms_per_step'], 'enc_t1', s['enc_t1_ms'], 'dec_t1', s['dec_t1_ms'])"
done
exit 0
