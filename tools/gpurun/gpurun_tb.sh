set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ba_gpu.py -q -m gpu -x > gpurun_out/diag_tests.log 2>&1 || { tail -40 gpurun_out/diag_tests.log; exit 1; }
tail -1 gpurun_out/diag_tests.log
bash gpurun_b.sh
