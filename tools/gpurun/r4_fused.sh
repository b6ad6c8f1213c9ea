# Round 4: the long reduce targets summed inside the reduce launch (last
# segment combines) vs the three-launch form (SFM_REDUCE_SPLIT=1).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/y_topcorner
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for v in fused split topsplit; do
  unset SFM_REDUCE_SPLIT SFM_BCR_TOP_SPLIT; [ $v = split ] && export SFM_REDUCE_SPLIT=1; [ $v = topsplit ] && export SFM_BCR_TOP_SPLIT=1; true
  timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$v N1 /" | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$v rank0-of-8 /" | tee -a "$OUT/ab.txt"
done
done
unset SFM_REDUCE_SPLIT SFM_BCR_TOP_SPLIT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p1" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p1" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_c4.csv"; rm -rf "$OUT/p1"
