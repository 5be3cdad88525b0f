#!/bin/bash
# Kernel statistics per library variant: rocprofv3 --kernel-trace --stats over bench.py (one
# config, no aux) once per grok_amd/libgrok_amd_<name>.so in $VARIANTS ("cur" = in-tree).
# Usage: VARIANTS="cur w" CFG=C3 bash tools/gpu_prof_variants.sh   (summaries: gpurun_out/pv_<v>_<cfg>.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
cfg=${CFG:-C2}
for v in ${VARIANTS:-cur}; do
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    rm -rf gpurun_out/pv_$v
    GROK_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$v -o run -- \
        python3 bench.py --config $cfg --steps 4 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/pv_${v}_$cfg.log 2>&1 || exit $?
    db=$(find gpurun_out/pv_$v -name '*.db' | head -1)
    python3 tools/prof_summary.py "$db" > gpurun_out/pv_${v}_$cfg.txt || exit $?
    grep -E "dwt|kernel " gpurun_out/pv_${v}_$cfg.txt
done
exit 0
