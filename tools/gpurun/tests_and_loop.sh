# GPU tier (all -m gpu tests, one pytest process) then the C5 loop profile.
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpurun/tests.sh
bash tools/gpurun/loop_prof.sh "${1:-loop}" "${2:-300}"
