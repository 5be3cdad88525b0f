#!/bin/bash
# Solo T1 decode check: parity tests (forced splits), then a C2 / C3 bench with decoder stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_t1solo.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/solo_test.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/solo_c2.log 2>&1 || exit $?
GK_T1DEC_SOLO=0 timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/nosolo_c2.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --config C3 --steps 3 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/solo_c3.log 2>&1 || exit $?
GK_T1DEC_SOLO=0 timeout -k 10 240 python bench.py --config C3 --steps 3 --warmup 1 --no-aux --no-cpu-baseline > gpurun_out/nosolo_c3.log 2>&1 || exit $?
