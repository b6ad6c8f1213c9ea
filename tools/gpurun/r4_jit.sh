# BA parity tests, BCR stamps and C4 A/B for library variants:
#   tools/gpurun/r4_jit.sh <tag> lib...   ("base" = in-tree)
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4j}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_ba_gpu.py tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_headline_gpu.py tests/test_seq_gpu.py"
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash tools/gpurun/bcr_stamps.sh "$@" | tee "$OUT/stamps.txt"
bash tools/gpurun/lib_ab.sh "$@" | tee "$OUT/ab.txt"
ARGS="--no-match --no-snavely --no-loop --no-pmc --no-filter --no-cpu-baseline --no-dense --no-radial3"
timeout -k 10 300 python -u bench.py --fake-world 8 --steps 20 $ARGS 2>&1 >/dev/null | grep "^\[bench\] BA:" | tee "$OUT/fake8.txt"
