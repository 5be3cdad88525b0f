cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in sold cur; do
  lib=$PWD/grok_amd/libgrok_amd.so; [ $v != cur ] && lib=$PWD/grok_amd/libgrok_amd_$v.so
  GROK_AMD_LIB=$lib GK_T1_STATS=2 timeout -k 10 200 python bench.py --config C3 --steps 1 --warmup 0 --no-aux --no-cpu-baseline > gpurun_out/ss_$v.log 2>&1 || exit $?
  echo $v; grep "t1dec solo\|t1dec timing" gpurun_out/ss_$v.log | tail -2
done
