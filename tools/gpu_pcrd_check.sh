#!/bin/bash
# rate-control tests, the C3 PCRD simulation checked against packet writes, the C3 host
# profile and a C2 bench line (one gpurun call; a failing step ends it)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pcrd_sim.py tests/test_gpu_rc_tiles.py tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_progression.py tests/test_gpu_tiles.py tests/test_gpu_modes.py \
    -x -q --timeout 300 > gpurun_out/t.log 2>&1 || exit $?
GK_T2_CHECK_SIM=1 timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 0 --no-aux --no-cpu-baseline \
    > gpurun_out/c3_check.log 2>&1 || exit $?
GK_PROFILE=1 timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-aux --no-cpu-baseline \
    > gpurun_out/c3_prof.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/c2.log 2>&1
