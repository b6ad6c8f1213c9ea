"""Per-LM-iteration kernel time by kernel family from rocprofv3 kernel_stats
CSVs (the BCR rows summed), for the round's profile summaries.
    python tools/kstat_brief.py kernel_stats_c4.csv [more.csv ...]"""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    # one Schur launch per LM iteration (the first pass of a solve included)
    iters = sum(int(r["Calls"]) for r in rows if r["Name"].startswith("void sfm::(anonymous namespace)::schur_kernel"))
    iters = max(iters, 1)
    fam = {}
    for r in rows:
        n = r["Name"]
        base = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
        key = base.split("(")[0].split("<")[0].split("::")[-1]
        fam[key] = fam.get(key, 0.0) + float(r["TotalDurationNs"]) / 1e3
    bcr = sum(v for k, v in fam.items() if k.startswith("bcr_"))
    tot = sum(fam.values())
    print(f"{path}: {iters} LM iterations; per iteration: all kernels {tot / iters:.1f} us, bcr_* {bcr / iters:.1f} us")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:16]:
        print(f"  {k:32s} {v / iters:8.1f} us")
