set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  N=$(echo $C | cut -d' ' -f1)
  timeout -k 10 900 rocprofv3 --pmc $C --kernel-include-regex "schur_kernel|match_top2_kernel|step_kernel|image_gram_kernel" --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc2/$N -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc2/$N.json 2> $R/gpurun_out/pmc2/$N.err || { tail -20 $R/gpurun_out/pmc2/$N.err; exit 1; }
  echo "pass $N done"
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc2 $R/gpurun_out/pmc2/pmc_summary.json
cat $R/gpurun_out/pmc2/pmc_summary.json
