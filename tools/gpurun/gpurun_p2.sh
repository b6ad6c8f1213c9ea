set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmcx
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex "schur_kernel" --kernel-trace --output-format csv -d $R/gpurun_out/pmcx/b -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match --no-snavely > $R/gpurun_out/pmcx/b.json 2> $R/gpurun_out/pmcx/b.err || { tail -20 $R/gpurun_out/pmcx/b.err; exit 1; }
