# Round 4: shard-sized step / Gram launches at N = 8 (step_kernel SPLIT lanes
# per point, gram_seg workgroups per image, one fill launch for the RCS clear).
# A/B against the previous kernels' shapes via SFM_STEP_SPLIT=1 SFM_GRAM_SEG=3.
#   tools/gpurun/r4_shard.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-k_shard}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh
cp gpurun_out/gputests.log "$OUT/gputests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for v in new old; do
  if [ $v = old ]; then export SFM_STEP_SPLIT=1 SFM_GRAM_SEG=3; else unset SFM_STEP_SPLIT SFM_GRAM_SEG; fi
  timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$v N1 /" | tee -a "$OUT/fake8.txt"
  timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$v rank0-of-8 /" | tee -a "$OUT/fake8.txt"
done
done
unset SFM_STEP_SPLIT SFM_GRAM_SEG
for sp in 2 4; do
  SFM_STEP_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/split$sp N1 /" | tee -a "$OUT/fake8.txt"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p8" -o f8 -- python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find "$OUT/p8" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fake8.csv"; rm -rf "$OUT/p8"
