# Quick state probe: the -m gpu tier, the C4 line with BCR phase stamps,
# rank 0's shard of an N=8 partition untraced (per-rank wall rate), and the
# 2-rank self-launch of bench.py on one device over the host all-reduce.
# Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-probe}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/gputests.log" 2>&1 || { tail -40 "$OUT/gputests.log"; exit 1; }
tail -2 "$OUT/gputests.log"
fi
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
SFM_BCR_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 $ARGS > "$OUT/c4_stamps.json" 2> "$OUT/c4_stamps.err" \
    || { tail -20 "$OUT/c4_stamps.err"; exit 1; }
grep -E "^\[bench\] BA|bcr stamps" "$OUT/c4_stamps.err" | tail -3
timeout -k 10 300 python -u bench.py --steps 5 $ARGS > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err"; exit 1; }
grep "^\[bench\] BA" "$OUT/c4.err"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 5 $ARGS > "$OUT/fake8.json" 2> "$OUT/fake8.err" \
    || { tail -20 "$OUT/fake8.err"; exit 1; }
grep "^\[bench\] BA" "$OUT/fake8.err"
SFM_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --allow-host-allreduce $ARGS \
    > "$OUT/n2.json" 2> "$OUT/n2.err" || { tail -30 "$OUT/n2.err"; exit 1; }
grep "^\[bench\] BA" "$OUT/n2.err" | head -2
python3 -c "import json; d=[json.loads(l) for l in open('$OUT/n2.json') if l.startswith('{')][-1]; print('N=2', d['n_gpus'], d['value'], d['config']['transport'], d['rmse_final'])"
