# A/B kernel times: rocprofv3 stats of the BA bench for the base library and each variant in $VARS
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for V in base $VARS; do
  if [ $V = base ]; then L=""; else L=$R/build/var_$V/libsfmcore.so; fi
  D=$R/gpurun_out/ab_$V
  rm -rf $D
  SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o k -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-match --no-snavely > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
  f=$(find $D -name "*kernel_stats.csv" | head -1)
  echo "== $V: $(python3 -c "import json; d=json.load(open('$D.json')); print(round(d['value'],1), 'it/s')")"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]: print('  ', r['Name'][:50].ljust(50), '%8.1f'%(float(r['AverageNs'])/1e3))
"
done
