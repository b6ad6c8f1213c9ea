set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -8 gpurun_out/bench.err
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1 -o bench -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  N=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "schur_kernel|match_top2_kernel|step_kernel|image_gram_kernel|bcr_level_kernel|casc_match_lds_kernel|casc_hash_kernel" --kernel-trace --output-format csv -d $R/gpurun_out/pmc3/$N -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc3/$N.json 2> $R/gpurun_out/pmc3/$N.err || { tail -20 $R/gpurun_out/pmc3/$N.err; exit 1; }
  echo "pass $N done"
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc3 $R/gpurun_out/pmc3/pmc_summary.json
