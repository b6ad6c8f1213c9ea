# Round-4 evidence: the whole GPU tier, then the default bench line with its
# rocprofv3 kernel stats (bench_prof.sh).   tools/gpurun/r4_tier.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4t}
mkdir -p gpurun_out/$TAG
bash tools/gpurun/tests.sh
cp gpurun_out/gputests.log gpurun_out/$TAG/gputests.log
bash tools/gpurun/bench_prof.sh $TAG
