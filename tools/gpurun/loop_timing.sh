# C5 loop with SFM_TIMING=1 (host phase times of every BA call), summed.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lt}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/loop_prof.py 300 > "$OUT/loop.json" 2> "$OUT/loop_plain.err" || { tail -20 "$OUT/loop_plain.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/loop.json').read().strip().splitlines()[-1]); print('plain', d['value'], d['seconds'], d['stage_seconds'])"
SFM_TIMING=1 timeout -k 10 300 python -u tools/loop_prof.py 300 > "$OUT/loop_t.json" 2> "$OUT/loop_timing.err" || { tail -20 "$OUT/loop_timing.err"; exit 1; }
python3 tools/phase_sum.py "$OUT/loop_timing.err" | head -24
