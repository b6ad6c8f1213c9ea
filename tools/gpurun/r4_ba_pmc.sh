# Round 4: SQ counters of the C4 BA kernels (Gram, step, Schur, reduce, BCR),
# two passes over a short C4 bench run.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/u_ba_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-match --no-snavely --no-loop --no-pmc --no-filter --no-dense --no-radial3 --no-cpu-baseline"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
C2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES"
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $C1 --output-format csv -d "$OUT/p1" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS) > "$OUT/p1.log" 2>&1
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $C2 --output-format csv -d "$OUT/p2" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS) > "$OUT/p2.log" 2>&1
ls -R "$OUT" | head -20
