set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${1:-r6dq}; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_ba_general_gpu.py tests/test_radial3.py > gpurun_out/${1:-r6dq}/tests.log 2>&1 || { tail -30 gpurun_out/${1:-r6dq}/tests.log; exit 1; }
tail -2 gpurun_out/${1:-r6dq}/tests.log
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for rep in 1 2; do timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera"; done
SFM_DENSE_STAMPS=1 timeout -k 10 300 python -u bench.py $BASE --no-radial3 2>&1 >/dev/null | grep "dense stamps" | tail -1
