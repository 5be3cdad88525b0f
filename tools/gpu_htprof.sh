cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
# C4 encode+decode once under rocprofv3 --kernel-trace --stats, for the in-tree library and
# grok_amd/libgrok_amd_<v>.so for each v in $HT_VARIANTS (k_ht_enc / k_ht_dec times).
for v in cur ${HT_VARIANTS:-}; do
  lib=$PWD/grok_amd/libgrok_amd.so; [ "$v" != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
  (cd /tmp && GROK_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ht_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config C4 --steps 1 --warmup 0 --no-aux --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/ht_$v.log 2>&1)
  rc=$?; echo "$v rc=$rc" >> gpurun_out/ht_steps.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0
