# GPU test tier: every -m gpu test in one process, each test under its own
# thread timeout, the whole step under a hard limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${1:+-k "$1"} \
    > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -5 gpurun_out/gputests.log
