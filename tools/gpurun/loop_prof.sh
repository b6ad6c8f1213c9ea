# C5 loop: host phase times of every BA call (SFM_TIMING=1) and a rocprofv3
# --kernel-trace --stats summary of the same loop.  Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-loop}
N=${2:-300}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py "$N" > "$OUT/loop.json" 2> "$OUT/loop_timing.err" || { tail -30 "$OUT/loop_timing.err"; exit 1; }
cat "$OUT/loop.json"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o loop -- \
    python3 "$GRAFT_REPO_ROOT/tools/loop_prof.py" "$N" > "$OUT/prof_loop.json" 2> "$OUT/prof_loop.err" || { tail -30 "$OUT/prof_loop.err"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:30]:
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(6), '%10.1f' % (float(r['AverageNs']) / 1e3), '%6.2f' % float(r['Percentage']))
PY
