# Round-4 batch 4: a dense-flow variant's parity tests (C5 loop vs the oracle,
# dense vs band, RADIAL3 per-camera) and the fixed-write-back loop A/B with
# the dense solve's kernel average.
#   tools/gpurun/r4_dflow.sh <tag> <variant.so>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4d}; V=${2:-vlib/libsfm_dflow.so}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_seq_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py"
SFMCORE_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_variant.log" 2>&1 || { tail -40 "$OUT/tests_variant.log"; exit 1; }
tail -1 "$OUT/tests_variant.log"
for rep in 1 2; do
for L in base $V; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_$(basename $L)_$rep.json" 2> /dev/null
    python3 -c "import json; d=json.loads(open('$OUT/loop_$(basename $L)_$rep.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['seconds'], d['stage_seconds']['ba'], d['ba_lm_iterations'])"
done
done
for L in base $V; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    d=$OUT/k_$(basename $L)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- python3 "$GRAFT_REPO_ROOT/tools/loop_prof.py" 300 fixed > /dev/null 2>&1)
    f=$(find "$d" -name '*kernel_stats.csv' | head -1)
    cp "$f" "$OUT/kernel_stats_loop_$(basename $L).csv"
    python3 - "$L" "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if "dense_flow" in r["Name"]:
        print("  %-24s dense_flow %5s calls %7.1f us" % (sys.argv[1][-24:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
    rm -rf "$d"
done
