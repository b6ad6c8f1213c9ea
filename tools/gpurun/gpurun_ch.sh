set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'iters', d['lm_iterations_per_solve'], 'schur ms', round(d['roofline']['per_launch_ms'],4))"
for C in 16 24 ; do
  echo "n_pt=62500 chunk $C:"
  SFM_BA_CHUNK_PTS=$C timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --n-pt 62500 --n-cam 125 2> gpurun_out/ch.err | python -c "$P"
done
for C in 32 48 ; do
  echo "n_pt=125000 chunk $C:"
  SFM_BA_CHUNK_PTS=$C timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --n-pt 125000 --n-cam 250 2> gpurun_out/ch.err | python -c "$P"
done
for C in 64 96 ; do
  echo "n_pt=250000 chunk $C:"
  SFM_BA_CHUNK_PTS=$C timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --n-pt 250000 --n-cam 500 2> gpurun_out/ch.err | python -c "$P"
done
echo "n_pt=250000 auto:"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match --no-snavely --n-pt 250000 --n-cam 500 2> gpurun_out/ch.err | python -c "$P"
