"""Per-LM-iteration kernel breakdown of the dense-S BA from a rocprofv3 kernel
trace: the dispatches between two consecutive dense_flow_kernel launches
(one iteration), summed by kernel over the last timed solves."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
fl = [i for i, k in enumerate(ks) if "dense_flow_kernel" in k[0]]
short = lambda n: n.replace("sfm::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]  # noqa: E731
pairs = list(zip(fl, fl[1:]))[-8:]
agg, walls = {}, []
for a, b in pairs:
    seg = ks[a:b]
    walls.append(seg[-1][2] - seg[0][1])
    for n, s, e in seg:
        t = agg.setdefault(short(n), [0, 0])
        t[0] += e - s
        t[1] += 1
n = len(pairs)
print(f"{n} iterations (dense_flow to dense_flow), wall {sum(walls) / n / 1e3:.1f} us each")
for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"  {k:48s} {c / n:5.1f} launches  {t / n / 1e3:8.1f} us")
