# Round 6: dense dataflow solve phase stamps on the C5 loop (chain per column,
# chain length and the substitution tail per solve).   tools/gpurun/r6_e.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6e}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SFM_DENSE_STAMPS=1 timeout -k 10 300 python -u tools/loop_prof.py 300 fixed > "$OUT/loop.json" 2> "$OUT/stamps.err" || { tail -20 "$OUT/stamps.err"; exit 1; }
grep "dense stamps" "$OUT/stamps.err" | tail -3
python3 - "$OUT/stamps.err" <<'PY'
import re, sys
ch = tl = n = 0
for l in open(sys.argv[1]):
    m = re.search(r"chain ([\d.]+) us, chain end to x_0 ([\d.]+) us over (\d+) solves", l)
    if m:
        k = int(m.group(3)); ch += float(m.group(1)) * k; tl += float(m.group(2)) * k; n += k
print("dataflow solves %d: chain %.1f us, tail %.1f us average" % (n, ch / max(n, 1), tl / max(n, 1)))
PY
