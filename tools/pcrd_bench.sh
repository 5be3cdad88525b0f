#!/bin/bash
# host-only PCRD timing harness (no GPU needed)
set -e
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip pcrd_bench.cpp -o /tmp/pcrd_bench -x none ../grok_amd/libgrok_amd.so -Wl,-rpath,$PWD/../grok_amd
GK_PROFILE=1 /tmp/pcrd_bench "$@"
