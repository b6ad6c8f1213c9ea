# C5 loop outcome (kept images, final BA RMSE) for several library builds.
set -e
cd "$GRAFT_REPO_ROOT"
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    r=$(timeout -k 10 200 python -u tools/loop_prof.py 300 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d.get('kept_images'), d.get('ba_lm_iterations'), d.get('final_ba'))" || echo failed)
    echo "$L: $r"
done
