set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex "schur_kernel|step_kernel|image_gram_kernel|bcr_level" --kernel-trace --output-format csv -d $R/gpurun_out/pmcx/a -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match --no-snavely > $R/gpurun_out/pmcx/a.json 2> $R/gpurun_out/pmcx/a.err || { tail -20 $R/gpurun_out/pmcx/a.err; exit 1; }
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$R/gpurun_out/pmcx/a/p_counter_collection.csv")))
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1][:30]
    d[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in d.items():
    print(n, {k: round(sum(v)/len(v)) for k, v in c.items()})
PY
