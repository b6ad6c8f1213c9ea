# Round-6 evidence for the committed tree: GPU tier, default bench line with
# rocprofv3 kernel stats (bench_prof.sh), rank 0 of N=8 untraced and its
# kernel stats.   tools/gpurun/r6_final.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-z_final}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh
cp gpurun_out/gputests.log "$OUT/gputests.log"
bash tools/gpurun/bench_prof.sh "$TAG"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/N1 /" | tee -a "$OUT/fake8.txt"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/rank0-of-8 /" | tee -a "$OUT/fake8.txt"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p8" -o f8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p8" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fake8.csv"; rm -rf "$OUT/p8" "$OUT/prof" "$OUT/prof_c4"
