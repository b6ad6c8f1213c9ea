# Per-step C5 loop traces for several library builds (diagnostic).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/ls
mkdir -p "$OUT"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 200 python -u tools/loop_steps.py 300 > "$OUT/$(basename $L).txt" 2>&1 || { tail -5 "$OUT/$(basename $L).txt"; exit 1; }
done
