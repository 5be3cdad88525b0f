#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_tiles.py -q -x -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for v in "0 4" "1 1" "1 2" "1 4" "1 8" "1 16"; do
  set -- $v
  GK_T1DEC=$1 GK_T1DEC_PARK=$2 GK_T1_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/bench_$1_$2.log 2>&1 || exit $?
done
