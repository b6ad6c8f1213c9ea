# General-point / dense-RCS GPU tests, then the dense-S and RADIAL3 lines and
# the dense-S kernel stats: tools/gpurun/dense_ab.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-da}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_ba_general_gpu.py tests/test_radial3.py tests/test_snavely.py tests/test_ba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 300 python -u tools/dense_prof.py 2>&1 | grep "dense-S"
bash tools/gpurun/dense_kstats.sh "${1:-da}"
