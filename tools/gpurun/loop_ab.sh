# BA + loop GPU tests, then the C5 loop in both write-back modes (plain runs
# and one SFM_TIMING run of the fixed mode, host phase sums).
#   tools/gpurun/loop_ab.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-la}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_ba_general_gpu.py tests/test_seq_gpu.py tests/test_radial3.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c3" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for mode in quirk fixed; do
timeout -k 10 300 python -u tools/loop_prof.py 300 $mode > "$OUT/loop_$mode.json" 2> "$OUT/loop_$mode.err"
python3 -c "import json; d=json.loads(open('$OUT/loop_$mode.json').read().strip().splitlines()[-1]); print('$mode', round(d['value'],2), 'img/s', round(d['seconds'],3), 's', {k: round(v,3) for k,v in d['stage_seconds'].items()}, d['ba_lm_iterations'], 'kept', d['kept_images'])"
done
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > /dev/null 2> "$OUT/timing_fixed.err"
python3 tools/phase_sum.py "$OUT/timing_fixed.err" > "$OUT/phase_sum_fixed.txt"
rm -f "$OUT/timing_fixed.err"
head -14 "$OUT/phase_sum_fixed.txt"
