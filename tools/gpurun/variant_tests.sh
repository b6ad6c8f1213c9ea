# Parity tests of library variants:
#   tools/gpurun/variant_tests.sh "<test files>" "<pytest -k expr or empty>" lib...
# ("base" = in-tree build); a failing variant stops the script.
set -e
cd "$GRAFT_REPO_ROOT"
FILES=$1; KEXPR=$2; shift 2
mkdir -p gpurun_out/vt
for L in "$@"; do
    if [ "$L" = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/$L; fi
    n=$(basename "$L")
    timeout -k 10 600 python -u -m pytest $FILES ${KEXPR:+-k "$KEXPR"} -m gpu -x -q --timeout 300 \
        --timeout-method thread > "gpurun_out/vt/$n.log" 2>&1 || { echo "$L: FAILED"; tail -30 "gpurun_out/vt/$n.log"; exit 1; }
    echo "$L: $(tail -1 gpurun_out/vt/$n.log)"
done
