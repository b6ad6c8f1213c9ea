set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_match_gpu.py -q -m gpu -x > gpurun_out/m_tests.log 2>&1 || { tail -40 gpurun_out/m_tests.log; exit 1; }
tail -1 gpurun_out/m_tests.log
timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/m_bench.json 2> gpurun_out/m_bench.err || { tail -20 gpurun_out/m_bench.err; exit 1; }
grep "match:" gpurun_out/m_bench.err
