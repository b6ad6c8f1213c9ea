# Round 4: the shard chunk length at N = 8 and N = 4 (SFM_BA_CHUNK_PTS).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/o_n8knobs
mkdir -p "$OUT"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
run() {  # tag, world, env...
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --fake-world $w --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$tag rank0-of-$w /" | tee -a "$OUT/pts.txt"
}
for rep in 1 2; do
  for p in 31 36 40 45 52; do run pts$p 8 SFM_BA_CHUNK_PTS=$p; done
  for p in 61 75 89 110; do run pts$p 4 SFM_BA_CHUNK_PTS=$p; done
  for p in 122 128; do run pts$p 2 SFM_BA_CHUNK_PTS=$p; done
done
