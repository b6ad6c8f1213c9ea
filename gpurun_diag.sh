set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_ba_gpu.py -q -m gpu -k "facade or c1" > gpurun_out/diag_tests.log 2>&1 || { tail -30 gpurun_out/diag_tests.log; exit 1; }
tail -2 gpurun_out/diag_tests.log
SFM_SCHUR_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match > gpurun_out/diag.json 2> gpurun_out/diag.err
grep -E "stamps|BA:" gpurun_out/diag.err | tail -4
