"""Print mean per-launch PMC counters per kernel from a rocprofv3 counter CSV.
usage: python tools/pmc_print.py <p_counter_collection.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1][:40]
    d[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in d.items():
    print(n, len(next(iter(c.values()))), {k: round(sum(v) / len(v)) for k, v in c.items()})
