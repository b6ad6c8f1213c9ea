set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_snavely.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-match --no-snavely 2> gpurun_out/q_b.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'schur ms', d['roofline']['per_launch_ms'], d['rmse_final'], d['lm_iterations_per_solve'])"
done
bash tools/gpurun/gpurun_prof.sh
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --fake-world 8 2> gpurun_out/fw.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fake world 8 value', d['value'], 'ms/step', d['ms_per_step'], 'iters', d['lm_iterations_per_solve'], 'schur ms', d['roofline']['per_launch_ms'])"
