cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_roi.py tests/test_gpu_progression.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; echo "tests rc=$?" >> gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/new.log 2>&1 && \
GROK_AMD_LIB=$PWD/grok_amd/libgrok_amd_old.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-aux --no-cpu-baseline > gpurun_out/old.log 2>&1
