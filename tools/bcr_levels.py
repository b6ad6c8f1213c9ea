"""Per-level duration of the BCR launches from a rocprofv3 kernel trace
(--kernel-trace --output-format csv: *_kernel_trace.csv): every RCS solve
launches (bcr_pack for a one-block band,) one bcr_level per level,
bcr_top_corner, bcr_back; the mean duration of each position in that
sequence is printed (us).  A sequence starts at the first BCR launch after
any other kernel.
    python tools/bcr_levels.py kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seqs, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if "bcr_" not in name:
        cur = None
        continue
    short = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0].split("<")[0].split("::")[-1]
    if cur is None:
        cur = []
        seqs.append(cur)
    if True:
        cur.append((short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                    int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
acc = defaultdict(list)
gaps = defaultdict(list)
for s in seqs:
    for k, (n, d, t0, t1) in enumerate(s):
        acc[(k, n)].append(d)
        if k:
            gaps[k].append((t0 - s[k - 1][3]) / 1e3)
tot = 0.0
for (k, n), v in sorted(acc.items()):
    m = sum(v) / len(v)
    tot += m
    g = sum(gaps[k]) / len(gaps[k]) if gaps[k] else 0.0
    print(f"{k:2d} {n:24s} {m:8.2f} us  (gap before {g:5.2f} us, {len(v)} solves)")
print(f"sum of means {tot:.1f} us per RCS solve")
