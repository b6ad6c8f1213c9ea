# Round 6: dense-S / RADIAL3 per-camera with the default library and the
# fewer-worker variants (tools/ab/w2.so, w4.so: half / a quarter of the task
# workers) -- is the dataflow solve bound by its workers or by its hand-offs?
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --steps 3 --warmup 1"
for v in "" tools/ab/w2.so tools/ab/w4.so ""; do
  echo "== ${v:-default}"
  SFMCORE_LIB=${v:+$GRAFT_REPO_ROOT/$v} timeout -k 10 300 python -u bench.py $BASE 2>&1 >/dev/null | grep -E "dense-S|per-camera"
done
