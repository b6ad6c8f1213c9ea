# Round 5, first look: GPU tier, the pivot-wave interference probe, BCR phase
# stamps at C4 and at rank 0 of N = 8.   tools/gpurun/r5_a.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5a}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpurun/tests.sh || { cp gpurun_out/gputests.log "$OUT/"; exit 1; }
cp gpurun_out/gputests.log "$OUT/gputests.log"
timeout -k 10 120 ./tools/probe/diag16_interf > "$OUT/interf.txt" 2>&1
cat "$OUT/interf.txt"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 $ARGS > /dev/null 2> "$OUT/stamps_c4.err"
grep "bcr stamps\|\[bench\] BA:" "$OUT/stamps_c4.err" | tail -3
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --fake-world 8 --steps 5 --warmup 1 $ARGS > /dev/null 2> "$OUT/stamps_f8.err"
grep "bcr stamps\|\[bench\] BA:" "$OUT/stamps_f8.err" | tail -3
