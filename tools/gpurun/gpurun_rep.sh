set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-match 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['per_launch_ms'])"
done
