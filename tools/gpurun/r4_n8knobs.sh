# Round 4: rank 0 of N = 8 (and N = 1) over Schur-side knobs: tile groups of
# 2 / 4 chunks (vlib/libsfm_g2.so, g4.so) and the shard's chunk length
# (SFM_BA_CHUNK_PTS), against the in-tree build.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/o_n8knobs
mkdir -p "$OUT"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
run() {  # tag, extra env..., then fake-world
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$tag rank0-of-8 /" | tee -a "$OUT/ab.txt"
}
for rep in 1 2; do
  run base SFM_NOTHING=1
  run g2 SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_g2.so
  run g4 SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_g4.so
  run pts20 SFM_BA_CHUNK_PTS=20
  run pts45 SFM_BA_CHUNK_PTS=45
  run pts64 SFM_BA_CHUNK_PTS=64
  run g4pts64 SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_g4.so SFM_BA_CHUNK_PTS=64
done
