#!/bin/bash
# DWT kernel statistics with components per workgroup (default) and one per workgroup
# (GK_DWT_CPW=1): rocprofv3 --kernel-trace --stats over bench.py per config in $CONFIGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CONFIGS:-C2}; do
for v in cpw one; do
    rm -rf gpurun_out/dab_$v
    extra=""; [ $v = one ] && extra="GK_DWT_CPW=1"
    env $extra timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dab_$v -o run -- \
        python3 bench.py --config $cfg --steps 4 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/dab_${v}_$cfg.log 2>&1 || exit $?
    db=$(find gpurun_out/dab_$v -name '*.db' | head -1)
    python3 tools/prof_summary.py "$db" > gpurun_out/dab_${v}_$cfg.txt || exit $?
    echo "== $v $cfg"; grep -E "dwt" gpurun_out/dab_${v}_$cfg.txt
done
done
exit 0
