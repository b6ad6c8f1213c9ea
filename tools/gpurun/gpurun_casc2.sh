set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cascade.py tests/test_mvg_io.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/casc_tests.log 2>&1 || { tail -60 gpurun_out/casc_tests.log; exit 1; }
tail -2 gpurun_out/casc_tests.log
for V in base $VARS; do
  if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/var_$V/libsfmcore.so; fi
  SFMCORE_LIB=$L timeout -k 10 300 python tools/casc_ab.py ${NF:-120} 2>&1 | grep -v amdgpu.ids
done
