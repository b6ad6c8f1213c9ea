set -e
cd $GRAFT_REPO_ROOT
P="import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'schur ms', round(d['roofline']['per_launch_ms'],4), d['lm_iterations_per_solve'], d['rmse_final'])"
for V in base sp5 sp6 base; do
  if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/var_$V/libsfmcore.so; fi
  echo -n "$V: "
  SFMCORE_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-match --no-snavely 2> /dev/null | python -c "$P"
done
