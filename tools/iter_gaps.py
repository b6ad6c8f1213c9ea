"""Where the GPU idles inside an LM solve, from a rocprofv3 kernel trace
(--kernel-trace --output-format csv: *_kernel_trace.csv).  Kernels are taken
in start order per queue-less timeline (all streams merged); the time between
one kernel's end and the next kernel's start that no other kernel covers is
idle.  Idle gaps are summed per (previous kernel -> next kernel) pair, and the
busy / idle split is printed per BA iteration (one finalize_kernel each).
    python tools/iter_gaps.py kernel_trace.csv [min_gap_us]"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0].split("<")[0].split("::")[-1]


rows = list(csv.DictReader(open(sys.argv[1])))
min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
pairs = defaultdict(lambda: [0, 0.0])
busy_end, prev = None, None
idle_total, n_fin = 0.0, 0
span0 = ev[0][0] if ev else 0
for t0, t1, n in ev:
    if busy_end is not None and t0 > busy_end:
        g = (t0 - busy_end) / 1e3
        if g >= min_gap and g < 2000.0:   # longer gaps: between solves / host phases
            pairs[(prev, n)][0] += 1
            pairs[(prev, n)][1] += g
            idle_total += g
    if busy_end is None or t1 > busy_end:
        busy_end, prev = t1, n
    if n == "finalize_kernel":
        n_fin += 1
print(f"{n_fin} finalize launches (LM iterations incl. iteration 0); idle gaps >= {min_gap} us and < 2 ms: "
      f"{idle_total:.1f} us in all, {idle_total / max(n_fin, 1):.1f} us per iteration")
for (a, b), (c, s) in sorted(pairs.items(), key=lambda x: -x[1][1])[:15]:
    print(f"  {a:28s} -> {b:28s} {c:6d} gaps {s / max(n_fin, 1):8.2f} us/iter  (mean {s / c:6.2f} us)")
