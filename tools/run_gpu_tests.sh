cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rsync.py tests/test_gpu_cdc.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?
tail -30 gpurun_out/gputests.log
exit $rc
