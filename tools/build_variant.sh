#!/bin/bash
# Build an A/B variant of libgrok_amd.so with one source replaced:
#   tools/build_variant.sh OUT.so SOURCE_NAME REPLACEMENT_FILE
# e.g. tools/build_variant.sh grok_amd/libgrok_amd_A.so gk_t1enc.hip /tmp/old_t1enc.hip
# Run with GROK_AMD_LIB=$PWD/OUT.so (grok_amd/__init__.py) to measure it.
set -e
cd "$(dirname "$0")/.."
OUT=$(realpath -m "$1"); NAME=$2; REPL=$(realpath "$3")
T=$(mktemp -d)
mkdir -p "$T/grok_amd/csrc"
cp -r include "$T/"
cp grok_amd/csrc/* "$T/grok_amd/csrc/"
cp "$REPL" "$T/grok_amd/csrc/$NAME"
cd "$T/grok_amd/csrc"
SRCS="gk_kernels.hip gk_dwt97.hip gk_dwt_any.hip gk_t1enc.hip gk_t1dec.hip gk_t1ms.hip gk_ht.hip gk_engine.cpp grk_shim.cpp"
for f in $SRCS; do
    hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $f -o ${f%.*}.o &
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $(for f in $SRCS; do echo ${f%.*}.o; done)
rm -rf "$T"
echo "$OUT"
