# Round 4: image Gram workgroups per image (SFM_GRAM_SEG 2..8 on a build with
# room for 8, vlib/libsfm_gseg8.so) at N = 1 and rank 0 of N = 8.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/cc_gseg
mkdir -p "$OUT"
export SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_gseg8.so
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for g in 3 4 6 8; do
  SFM_GRAM_SEG=$g timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/gseg$g N1 /" | tee -a "$OUT/ab.txt"
done
for g in 2 3 4; do
  SFM_GRAM_SEG=$g timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/gseg$g rank0-of-8 /" | tee -a "$OUT/ab.txt"
done
done
