#!/bin/bash
# GPU-box check for one gpurun call: parity tests, the C3 rate-control simulation checked
# against real packet writes (GK_T2_CHECK_SIM), the C3 PCRD host profile and the C2 bench.
# Each GPU step has its own time limit; a failing step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
TESTSEL="${TESTSEL:-tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tiles.py}" PYTEST_ARGS=-x \
    bash tools/gpu_run.sh test || exit $?
grep -q "failed\|error" gpurun_out/pytest_gpu.log && exit 1
GK_T2_CHECK_SIM=1 timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 0 --no-aux --no-cpu-baseline \
    > gpurun_out/c3_check.log 2>&1 || exit $?
GK_PROFILE=1 timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --no-aux --no-cpu-baseline \
    > gpurun_out/c3_prof.log 2>&1 || exit $?
LANES_AB="64:64" bash tools/lanes_ab.sh || exit $?
exit 0
