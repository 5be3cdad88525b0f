#!/bin/bash
# Host-only PCRD timing on the GPU box's CPU share (tools/pcrd_bench.cpp on the C3 pass dump,
# gpurun_out/c3.pass.gz from tools/gpu_c3dump.sh).  No GPU call.  Usage: bash tools/gpu_pcrd_host.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
gunzip -c scratch/c3.pass.gz > /tmp/c3.pass || exit 1
for v in ${PCRD_VARIANTS:-/tmp/pcrd_bench}; do
  echo "== $v"
  (cd tools && GK_PROFILE=1 timeout -k 10 120 "bin/$(basename $v)" 8192 /tmp/c3.pass) 2>&1 | tail -14 || exit $?
done
