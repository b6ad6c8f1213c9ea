# Multi-rank rehearsal on one GPU: the memory-cache test, rank 0's shard of an
# N=8 landmark partition under rocprofv3 (per-rank kernel times), and a 2-rank
# run of bench.py (two processes on one device over the host gloo all-reduce;
# RCCL needs distinct devices).  Outputs under gpurun_out/<tag>/.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-shard}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q -k memory_cache --timeout 200 --timeout-method thread > "$OUT/cache_test.log" 2>&1 || { tail -30 "$OUT/cache_test.log"; exit 1; }
tail -2 "$OUT/cache_test.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof8" -o s8 -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --fake-world 8 --steps 5 $ARGS > "$OUT/fake8.json" 2> "$OUT/fake8.err" || { tail -20 "$OUT/fake8.err"; exit 1; }
f=$(find "$OUT/prof8" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats_fake8.csv"
rm -rf "$OUT/prof8"
grep "^\[bench\] BA" "$OUT/fake8.err"
cd "$GRAFT_REPO_ROOT"
SFM_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --allow-host-allreduce $ARGS \
    > "$OUT/n2.json" 2> "$OUT/n2.err" || { tail -20 "$OUT/n2.err"; exit 1; }
grep "^\[bench\] BA" "$OUT/n2.err" | head -2
python3 -c "import json,sys; d=json.load(open('$OUT/n2.json')); print('N=2', d['value'], d['config']['transport'], d['rmse_final'])"
