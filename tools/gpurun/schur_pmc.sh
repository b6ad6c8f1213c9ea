# Instruction mix of the Schur kernel (C4 plan, two solves): two --pmc passes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-spmc}
mkdir -p "$OUT"
cd /tmp
n=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES" \
         "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "schur_kernel|image_gram|step_kernel" --output-format csv \
      -d "$OUT/p$n" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --pmc-child > "$OUT/p$n.log" 2>&1 || { tail -5 "$OUT/p$n.log"; exit 1; }
  f=$(find "$OUT/p$n" -name '*counter_collection.csv' | head -1)
  cp "$f" "$OUT/counters_$n.csv"; rm -rf "$OUT/p$n"
done
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/counters_*.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1][:40] + ("<5>" if "ILi5E" in r["Kernel_Name"] or ", 5," in r["Kernel_Name"] else "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):14.4g}  n={len(v)}")
PY
