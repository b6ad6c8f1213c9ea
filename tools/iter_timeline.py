"""Per-iteration timeline of the C4 BA from a rocprofv3 kernel trace: the
last timed solve's dispatches in order with their durations and the idle gap
before each, plus totals (kernel time vs wall)."""
import csv
import gzip
import sys

f = sys.argv[1]
rows = list(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# the timed solves: schur launches mark iterations; take the span from the
# last gram_rescale (start of the last solve) to the end of the trace's BA part
starts = [i for i, k in enumerate(ks) if "gram_rescale" in k[0]]
if len(starts) < 2:
    print("no solves found")
    sys.exit(0)
# the timed solves run back to back: the shortest span between two starts
a, b = min(zip(starts, starts[1:]), key=lambda ab: ks[ab[1]][1] - ks[ab[0]][1])
seg = ks[a:b]
short = lambda n: n.replace("sfm::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
tot_k = sum(e - s for _, s, e in seg)
wall = seg[-1][2] - seg[0][1]
print(f"one solve: {len(seg)} dispatches, kernel {tot_k / 1e3:.1f} us, wall {wall / 1e3:.1f} us, "
      f"idle {(wall - tot_k) / 1e3:.1f} us")
agg = {}
prev = None
for n, s, e in seg:
    g = 0 if prev is None else s - prev
    k = short(n)
    d = agg.setdefault(k, [0, 0, 0])
    d[0] += 1
    d[1] += e - s
    d[2] += max(g, 0)
    prev = e
print(f"{'kernel':48s} {'calls':>5s} {'busy us':>9s} {'gap-before us':>14s}")
for k, (c, t, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:48s} {c:5d} {t / 1e3:9.1f} {g / 1e3:14.1f}")
print("\nsequence (first 60):")
prev = None
for n, s, e in seg[:60]:
    print(f"  gap {0 if prev is None else (s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:7.1f}  {short(n)}")
    prev = e
