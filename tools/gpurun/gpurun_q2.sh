set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_snavely.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match 2> gpurun_out/q_b.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'schur ms', d['roofline']['per_launch_ms'], 'frac', d['roofline']['frac'], d['rmse_final'], d['lm_iterations_per_solve']); s=d['ba_snavely']; print('snavely', s['value'], s['roofline']['per_launch_ms'], s['rmse_final'], s['lm_iterations_per_solve'])"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex "schur_kernel" --kernel-trace --output-format csv -d $R/gpurun_out/pmcx/b -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match --no-snavely > $R/gpurun_out/pmcx/b.json 2> $R/gpurun_out/pmcx/b.err || { tail -20 $R/gpurun_out/pmcx/b.err; exit 1; }
