#!/bin/bash
# Decoder step-group size A/B: the in-tree library (T1DEC_UNROLL 12) against _u10 / _u16 variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in 1 2; do
  for v in cur u10 u16; do
    lib=$PWD/grok_amd/libgrok_amd.so
    [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
    GROK_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/ab_${v}_$i.log 2>&1 || exit $?
  done
done
