set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in ${VARS:-base}; do
  if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/var_$V/libsfmcore.so; fi
  SFMCORE_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-match 2> gpurun_out/var_$V.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['per_launch_ms'],4), d['rmse_final'])"
done
