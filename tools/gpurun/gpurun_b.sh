set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match 2> gpurun_out/diagb.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['per_launch_ms'], d['roofline']['frac'], d['rmse_final'], d['lm_iterations_per_solve'])"
bash tools/gpurun/gpurun_prof.sh
