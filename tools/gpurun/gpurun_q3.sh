set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_snavely.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely 2> gpurun_out/q_b.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'schur ms', d['roofline']['per_launch_ms'], d['rmse_final'], d['lm_iterations_per_solve'])"
SFM_BCR_STAMPS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-match --no-snavely > gpurun_out/diag_bs.json 2> gpurun_out/diag_bs.err
grep -E "stamps" gpurun_out/diag_bs.err | tail -1
