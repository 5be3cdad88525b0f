#!/bin/bash
# A/B of library variants: bench.py (C2, no aux) once per grok_amd/libgrok_amd_<name>.so in
# $VARIANTS ("cur" = the in-tree library).  Logs: gpurun_out/var_<name>.log
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${VARIANTS:-cur}; do
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    GROK_AMD_LIB=$lib timeout -k 10 240 python bench.py --steps 8 --warmup 2 --no-aux --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$v.log 2>&1 || exit $?
done
exit 0
