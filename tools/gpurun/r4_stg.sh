# Round-4: pinned-staging plan uploads (variant) -- the C5 loop's BA stage
# A/B (fixed write-back, twice each) and the variant's phase sums.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4stg}; V=${2:-vlib/libsfm_stg.so}
mkdir -p "$OUT"
export TMPDIR=/tmp
SFMCORE_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 600 python -u -m pytest tests/test_seq_gpu.py tests/test_ba_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests_variant.log" 2>&1 || { tail -40 "$OUT/tests_variant.log"; exit 1; }
tail -1 "$OUT/tests_variant.log"
for rep in 1 2; do
for L in base $V; do
    unset SFMCORE_LIB; [ "$L" != base ] && export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L
    timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_$(basename $L)_$rep.json" 2> /dev/null
    python3 -c "import json; d=json.loads(open('$OUT/loop_$(basename $L)_$rep.json').read().strip().splitlines()[-1]); print('$L', d['value'], d['seconds'], d['stage_seconds']['ba'], d['ba_lm_iterations'])"
done
done
export SFMCORE_LIB=$GRAFT_REPO_ROOT/$V
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > /dev/null 2> "$OUT/timing.err"
python3 tools/phase_sum.py "$OUT/timing.err" | head -30 > "$OUT/phase_sum_fixed.txt"; rm -f "$OUT/timing.err"
head -20 "$OUT/phase_sum_fixed.txt"
