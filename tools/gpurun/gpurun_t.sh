set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_tests.log 2>&1 || { tail -40 gpurun_out/t_tests.log; exit 1; }
tail -3 gpurun_out/t_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match 2> gpurun_out/q_b.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'schur ms', d['roofline']['per_launch_ms'], 'frac', d['roofline']['frac'], d['rmse_final'], d['lm_iterations_per_solve'])"
