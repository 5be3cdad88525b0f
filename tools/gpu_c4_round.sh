#!/bin/bash
# C4 after an HT change: HT/full-size GPU tests, bench line, kernel stats + PMC traffic
# (tools/gpu_profile_all.sh), SQ counters (tools/sq_counters2.sh).  Usage: bash tools/gpu_c4_round.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-c4}
bash tools/gpu_suite.sh ${tag} tests/test_gpu_ht.py tests/test_gpu_ht97.py tests/test_gpu_fullsize.py tests/test_gpu_modes.py || exit $?
SKIP_SUITE=1 bash tools/gpu_check_quick.sh ${tag} C4 || exit $?
CONFIGS=C4 bash tools/gpu_profile_all.sh ${tag} || exit $?
PROF_ARGS="--config C4" bash tools/sq_counters2.sh || exit $?
exit 0
