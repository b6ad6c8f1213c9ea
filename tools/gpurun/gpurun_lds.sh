set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lds
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-include-regex "${KRE:-schur_kernel}" --kernel-trace --output-format csv -d $R/gpurun_out/lds -o p -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-match > $R/gpurun_out/lds/b.json 2> $R/gpurun_out/lds/b.err || { tail -20 $R/gpurun_out/lds/b.err; exit 1; }
python3 - <<'PY'
import csv, collections, os
R=os.environ['GRAFT_REPO_ROOT']
per=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(R+'/gpurun_out/lds/p_counter_collection.csv')):
    name=r["Kernel_Name"].replace("(anonymous namespace)::","").replace("void ","").split("(")[0].split("::")[-1]
    per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,d in per.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c,v in sorted(d.items())))
PY
