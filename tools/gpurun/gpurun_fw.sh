set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in 8; do
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --fake-world $W 2> gpurun_out/fw.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fake world $W value', d['value'], 'ms/step', d['ms_per_step'], 'iters', d['lm_iterations_per_solve'], 'schur ms', d['roofline']['per_launch_ms'])"
grep plan: gpurun_out/fw.err
done
D=$GRAFT_REPO_ROOT/gpurun_out/prof_fw
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o fw -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-match --no-snavely --fake-world 8 > $GRAFT_REPO_ROOT/gpurun_out/prof_fw.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_fw.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_fw.err; exit 1; }
f=$(find $D -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:25]: print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), '%10.1f'%(float(r['AverageNs'])/1e3), '%6.2f'%float(r['Percentage']))
"
