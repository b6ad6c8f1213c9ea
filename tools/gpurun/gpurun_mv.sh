set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in base u2w3 u2w4 u4w2; do
  if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/build/var_$V/libsfmcore.so; fi
  echo "== $V"
  SFMCORE_LIB=$L timeout -k 10 300 python tools_match_probe.py 200 2>/dev/null | tail -1
done
