# Round 6: the product-term reduce's batch size (SFM_PTB variants
# tools/ab/ptb8.so, ptb12.so against the default 16): dense-S and RADIAL3
# per-camera lines, then the dense tests on the best-looking variant is left
# to a separate run.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for v in "" tools/ab/ptb8.so tools/ab/ptb12.so "" tools/ab/ptb8.so tools/ab/ptb12.so; do
  echo "== ${v:-default}"
  SFMCORE_LIB=${v:+$GRAFT_REPO_ROOT/$v} timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera"
done
