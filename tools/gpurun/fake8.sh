set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f8
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f8/tests.log 2>&1 || { tail -30 gpurun_out/f8/tests.log; exit 1; }
tail -1 gpurun_out/f8/tests.log
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --steps 10 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA"
for cp in 0 16; do
  SFM_BA_CHUNK_PTS=$( [ $cp = 0 ] && echo "" || echo $cp ) timeout -k 10 300 python -u bench.py --fake-world 8 --steps 10 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/chunk=$cp /"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/f8/p -o f8 -- python3 $GRAFT_REPO_ROOT/bench.py --fake-world 8 --steps 10 $ARGS > /dev/null 2>&1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/f8/p -name "*kernel_stats.csv" | head -1); cp $f $GRAFT_REPO_ROOT/gpurun_out/f8/kernel_stats_fake8.csv; rm -rf $GRAFT_REPO_ROOT/gpurun_out/f8/p
