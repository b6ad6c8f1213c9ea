# Instruction mix and MFMA busy of match_top2_kernel (tools/match_pmc_child.py):
# two --pmc passes, each in its own run.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-mpmc}
mkdir -p "$OUT"
cd /tmp
n=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES" \
         "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "match_top2" --output-format csv \
      -d "$OUT/p$n" -o p -- python3 "$GRAFT_REPO_ROOT/tools/match_pmc_child.py" > "$OUT/p$n.log" 2>&1 || { tail -5 "$OUT/p$n.log"; exit 1; }
  f=$(find "$OUT/p$n" -name '*counter_collection.csv' | head -1)
  cp "$f" "$OUT/counters_$n.csv"; rm -rf "$OUT/p$n"
done
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/counters_*.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} last dispatch {v[-1]:14.4g}  n={len(v)}")
PY
