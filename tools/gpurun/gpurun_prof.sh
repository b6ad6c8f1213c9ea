set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
D=$GRAFT_REPO_ROOT/gpurun_out/prof_ba
rm -rf $D
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-match --no-snavely > $GRAFT_REPO_ROOT/gpurun_out/prof_ba.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_ba.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_ba.err; exit 1; }
f=$(find $D -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:25]: print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), '%10.1f'%(float(r['AverageNs'])/1e3), '%6.2f'%float(r['Percentage']))
"
