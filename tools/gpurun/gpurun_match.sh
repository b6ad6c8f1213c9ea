set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_match_gpu.py -x -q -m gpu > gpurun_out/match_tests.log 2>&1 || { tail -30 gpurun_out/match_tests.log; exit 1; }
tail -3 gpurun_out/match_tests.log
timeout -k 10 300 python tools_match_probe.py 96 > gpurun_out/match_probe.log 2>&1
cat gpurun_out/match_probe.log
