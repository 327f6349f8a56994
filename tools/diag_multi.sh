cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 170 python -u -m pytest tests/test_gpu_multi.py -x -v -rf --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/diag_multi.log 2>&1
echo "rc=$?" >> gpurun_out/diag_multi.log
