#!/bin/bash
# Host-only PCRD timing of one pcrd_bench binary (tools/bin/pcrd_bench) under several environment
# settings, on the GPU box's CPU share; no GPU call.  Usage: RUNS="name:VAR=VAL,VAR=VAL ..." bash tools/gpu_pcrd_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
gunzip -c scratch/c3.pass.gz > /tmp/c3.pass || exit 1
for rep in 1 2; do
for r in $RUNS; do
  name=${r%%:*}; vars=${r#*:}
  envs=(GK_PROFILE=1)
  [ "$vars" != "$name" ] && IFS=',' read -ra kv <<< "$vars" && envs+=("${kv[@]}")
  out=$(cd tools && env "${envs[@]}" timeout -k 10 120 bin/pcrd_bench 8192 /tmp/c3.pass 2>&1) || { echo "$out" | tail -5; exit 1; }
  par=$(echo "$out" | grep -o "parallel steps [0-9.]* ms" | awk '{print $3}' | sort -n | head -1)
  al=$(echo "$out" | grep -o "^allocate [0-9.]* ms" | awk '{print $2}' | sort -n | head -1)
  h=$(echo "$out" | grep -o "hash [0-9a-f]*" | tail -1)
  echo "$name: min parallel steps $par ms, min allocate $al ms, $h"
done
done
