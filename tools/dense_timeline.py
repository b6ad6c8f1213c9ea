#!/usr/bin/env python3
"""One dense RCS factorisation's timeline from a rocprofv3 kernel trace:
the launches from a dense_panel_kernel to the next dense_back_all_kernel
(the launch-chain path), grouped by kind -- panel, narrow update (grid below
the trailing update's), trailing update -- with their busy time and the
gaps between them.   python tools/dense_timeline.py kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"]  # noqa: E731
solves, cur = [], None
for r in rows:   # from the first panel launch (round 6: no pack launch) to the back substitution
    n = name(r)
    if cur is None and "dense_panel_kernel" in n:
        cur = [r]
    elif cur is not None:
        cur.append(r)
        if "dense_back_all_kernel" in n:
            solves.append(cur)
            cur = None
print(f"{len(solves)} dense factorisations in the trace")
for s in solves[-2:]:
    t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
    busy = {}
    cnt = {}
    gaps = 0
    prev_end = None
    panels = 0
    for r in s:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = name(r)
        k = "panel" if "panel" in n else "update" if "update" in n else "back" if "back" in n else "pack" if "pack" in n else n[:40]
        panels += k == "panel"
        if k == "update":   # groups of 4 columns: panel, narrow, ..., the 4th panel, trailing
            k = "update (trailing)" if panels % 4 == 0 else "update (narrow)"
        busy[k] = busy.get(k, 0) + (b - a)
        cnt[k] = cnt.get(k, 0) + 1
        if prev_end is not None and a > prev_end:
            gaps += a - prev_end
        prev_end = max(prev_end or 0, b)
    print(f"span {(t1 - t0) / 1e3:.1f} us, kernels {sum(busy.values()) / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us")
    for k in sorted(busy, key=lambda k: -busy[k]):
        print(f"  {k:22s} {cnt[k]:4d} launches {busy[k] / 1e3:9.1f} us  ({busy[k] / cnt[k] / 1e3:.1f} us each)")
