# BCR change check: BA parity tests, then C4 and rank 0's shard of N=8,
# in-tree build against an environment variant (A/B on one box).
#   tools/gpurun/bcr_ab.sh <tag> [ENV=VALUE for the B arm]
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bcr}
BENV=${2:-SFM_NOTHING=1}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_ba_gpu.py tests/test_headline_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_seq_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c3 and not full_300" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/A   /"
env $BENV timeout -k 10 300 python -u bench.py --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/B   /"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/A8  /"
env $BENV timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | sed "s/^/B8  /"
done
