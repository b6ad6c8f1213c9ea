# Round 6: landmark-shard chunk target A/B (in-tree 1850 vs variants) at
# N = 1 and --fake-world 2 / 4 / 8, alternating, two reps.
#   tools/gpurun/r6_i.sh <tag> variant.so...
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6i}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BASE="--no-match --no-snavely --no-pmc --no-filter --no-cpu-baseline --no-loop --no-dense --no-radial3 --steps 20 --warmup 3"
for rep in 1 2; do
  for W in 1 2 4 8; do
    for v in in-tree "$@"; do
      L=""; [ "$v" != in-tree ] && L="$GRAFT_REPO_ROOT/$v"
      FW=""; [ "$W" != 1 ] && FW="--fake-world $W"
      SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py $BASE $FW > "$OUT/b_${W}_$(basename $v).json" 2> "$OUT/b_${W}_$(basename $v).err"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'N', sys.argv[3], round(d['value'],1), d['unit'])" "$OUT/b_${W}_$(basename $v).json" "$v" "$W" | tee -a "$OUT/ab.txt"
    done
  done
done
