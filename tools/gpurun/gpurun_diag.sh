set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ba_gpu.py -q -m gpu -x > gpurun_out/diag_tests.log 2>&1 || { tail -40 gpurun_out/diag_tests.log; exit 1; }
tail -1 gpurun_out/diag_tests.log
for SUB in 0; do
SFM_SCHUR_SUB=$SUB SFM_SCHUR_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match > gpurun_out/diag_s.json 2> gpurun_out/diag_s.err
grep -E "stamps" gpurun_out/diag_s.err | tail -1
SFM_SCHUR_SUB=$SUB timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match 2> gpurun_out/diagb.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sub $SUB', d['value'], d['ms_per_step'], d['roofline']['per_launch_ms'], d['roofline']['frac'])"
done
