set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cascade.py tests/test_match_gpu.py tests/test_mvg_io.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/casc_tests.log 2>&1 || { tail -60 gpurun_out/casc_tests.log; exit 1; }
tail -5 gpurun_out/casc_tests.log
