set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SFM_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --n-pt 50000 --n-cam 200 --match-frames 16 > gpurun_out/mr.json 2> gpurun_out/mr.err || { tail -30 gpurun_out/mr.err; exit 1; }
grep -E "bench|RCCL|fall" gpurun_out/mr.err | tail -8
cat gpurun_out/mr.json
