#!/bin/bash
# GPU test suite on the box: pytest -m gpu (every test, per-test time limit), one log under
# gpurun_out/.  Usage: bash tools/gpu_suite.sh TAG [pytest args...]
tag=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider "${@:-tests}" \
    > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/${tag}_pytest_gpu.log
exit $rc
