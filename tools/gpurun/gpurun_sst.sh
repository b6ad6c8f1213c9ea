set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SFM_SCHUR_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match > gpurun_out/diag_s.json 2> gpurun_out/diag_s.err
grep -E "stamps" gpurun_out/diag_s.err | tail -1
