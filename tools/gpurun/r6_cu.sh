# Round 6: the dataflow schedule's chain-step weight (SFM_DF_CHAIN_UNITS
# variants tools/ab/cu5.so, cu10.so, cu40.so against the default 20):
# dense-S and RADIAL3 per-camera lines.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for v in "" tools/ab/cu5.so tools/ab/cu10.so tools/ab/cu40.so ""; do
  echo "== ${v:-default}"
  SFMCORE_LIB=${v:+$GRAFT_REPO_ROOT/$v} timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera"
done
