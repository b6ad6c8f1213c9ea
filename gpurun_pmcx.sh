set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for C in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32" "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS SQ_LDS_ADDR_CONFLICT SQ_INSTS_MFMA" "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "schur_kernel|step_kernel|image_gram_kernel|bcr_level_kernel" --kernel-trace --output-format csv -d $R/gpurun_out/pmcx/p$i -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match > $R/gpurun_out/pmcx/p$i.json 2> $R/gpurun_out/pmcx/p$i.err || { tail -20 $R/gpurun_out/pmcx/p$i.err; exit 1; }
  echo "pass $i done"
done
