# Dense dataflow solve A/B: dense + loop GPU tests, then the C5 loop (fixed
# write-back) with the dataflow kernel and with the launch chain
# (SFM_DENSE_LAUNCHES=1).   tools/gpurun/flow_ab.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-fa}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_ba_gpu.py tests/test_seq_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for v in flow launches; do
  if [ $v = launches ]; then export SFM_DENSE_LAUNCHES=1; fi
  timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop_$v.json" 2> "$OUT/loop_$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/loop_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), 'img/s', round(d['seconds'],3), 's', {k: round(v,3) for k,v in d['stage_seconds'].items()}, d['ba_lm_iterations'], 'kept', d['kept_images'])"
done
unset SFM_DENSE_LAUNCHES
timeout -k 10 300 python -u tools/dense_prof.py 2>&1 | grep "dense-S"
SFM_DENSE_FLOW_MAX_NT=1000 timeout -k 10 300 python -u tools/dense_prof.py 2>&1 | grep "dense-S" | sed 's/^/flow all nt: /'
