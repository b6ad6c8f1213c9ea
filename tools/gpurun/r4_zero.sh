# Round 4: rank 0 of N = 8 with the zero list cleared inside the reduce launch
# vs the old whole-RCS fill before it (SFM_RCS_FILL=1).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/bb_zero
mkdir -p "$OUT"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
for rep in 1 2; do
for v in zero fill; do
  unset SFM_RCS_FILL; [ $v = fill ] && export SFM_RCS_FILL=1; true
  timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/$v rank0-of-8 /" | tee -a "$OUT/ab.txt"
done
done
