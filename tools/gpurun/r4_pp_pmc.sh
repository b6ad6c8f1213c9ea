# Round 4: SQ counters of the exact matcher, in-tree vs the ping-pong build
# (vlib/libsfm_pp.so), on tools/match_pmc_child.py (2016 C3-shaped pairs).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/s_pp_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in base pp; do
  if [ $v = base ]; then unset SFMCORE_LIB; else export SFMCORE_LIB=$GRAFT_REPO_ROOT/vlib/libsfm_pp.so; fi
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/$v/p1" -o p -- python3 "$GRAFT_REPO_ROOT/tools/match_pmc_child.py") > "$OUT/$v.p1.log" 2>&1
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C2 -d "$OUT/$v/p2" -o p -- python3 "$GRAFT_REPO_ROOT/tools/match_pmc_child.py") > "$OUT/$v.p2.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in ("base", "pp"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(os.path.join(out, v, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "match_top2" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(v, {k: round(agg[k] / max(n[k], 1)) for k in sorted(agg)})
PY
