# Round 4: reduce_kernel with 1 / 2 / 4 waves per target (SFM_REDUCE_WAVES),
# N = 1 and rank 0 of N = 8, after the GPU tier.   tools/gpurun/r4_redw.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-m_redw}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh
cp gpurun_out/gputests.log "$OUT/gputests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for w in 1 2 4; do
  SFM_REDUCE_WAVES=$w timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/w$w N1 /" | tee -a "$OUT/ab.txt"
  SFM_REDUCE_WAVES=$w timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/w$w rank0-of-8 /" | tee -a "$OUT/ab.txt"
done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p8" -o f8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p8" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fake8.csv"; rm -rf "$OUT/p8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p1" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p1" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_c4.csv"; rm -rf "$OUT/p1"
