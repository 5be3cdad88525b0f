#!/bin/bash
# C3 encode once with GK_DUMP_PASSES: the pass records tools/pcrd_bench replays on the host.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
GK_DUMP_PASSES=gpurun_out/c3.pass timeout -k 10 240 python bench.py --config C3 --steps 1 --warmup 0 \
    --no-aux --no-cpu-baseline > gpurun_out/c3dump.log 2>&1 || exit $?
gzip -1 -f gpurun_out/c3.pass
