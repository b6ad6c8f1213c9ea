set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_ba_gpu.py -x -q -m gpu -k "${K:-.}" > gpurun_out/ba_tests.log 2>&1 || { tail -60 gpurun_out/ba_tests.log; exit 1; }
tail -5 gpurun_out/ba_tests.log
