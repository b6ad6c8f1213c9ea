"""Sum SFM_TIMING phase lines over a run: python tools/phase_sum.py timing.err"""
import re
import sys
from collections import defaultdict

tot = defaultdict(float)
cnt = defaultdict(int)
for line in open(sys.argv[1]):
    m = re.match(r"\[timing\] (\S+): (.*)", line)
    if not m:
        continue
    cnt[m.group(1)] += 1
    for k, v in re.findall(r"(\w+) ([0-9.]+) ms", m.group(2)):
        tot[(m.group(1), k)] += float(v)
for (f, k), v in sorted(tot.items(), key=lambda x: -x[1]):
    if v > 20:
        print(f"{f:28s} {k:16s} {v:9.1f} ms over {cnt[f]} calls")
