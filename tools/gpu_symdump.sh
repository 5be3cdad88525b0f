#!/bin/bash
# C2 encode once with GK_DUMP_SYMS: per-block MQ decision counts and bit-planes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
GK_DUMP_SYMS=gpurun_out/c2.syms timeout -k 10 240 python bench.py --steps 1 --warmup 0 \
    --no-aux --no-cpu-baseline > gpurun_out/symdump.log 2>&1
