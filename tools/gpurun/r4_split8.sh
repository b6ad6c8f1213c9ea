# Round 4: step-kernel lanes per point at rank 0 of N = 8 after the 1600-chunk
# target (~40-point chunks: 2 lanes = two waves per workgroup).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/gg_split8
mkdir -p "$OUT"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for sp in 1 2; do
  SFM_STEP_SPLIT=$sp timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/split$sp rank0-of-8 /" | tee -a "$OUT/ab.txt"
  SFM_STEP_SPLIT=$sp timeout -k 10 300 python -u bench.py --fake-world 4 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/split$sp rank0-of-4 /" | tee -a "$OUT/ab.txt"
done
done
