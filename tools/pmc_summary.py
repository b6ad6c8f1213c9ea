"""Summarise rocprofv3 --pmc passes into profiles/<round>/pmc_summary.json.

Per kernel: mean FETCH_SIZE / WRITE_SIZE per launch (rocprofv3 reports KiB),
the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the
bytes of wide coalesced reads -> doubled), and SQ_VALU_MFMA_BUSY_CYCLES when
that pass exists.  bench.py reads the result for roofline.traffic.

usage: python tools/pmc_summary.py <pmc dir with FETCH_SIZE/ WRITE_SIZE/ ...> <out.json>
"""
import collections
import csv
import json
import os
import sys


def main(src, out):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, d in per.items():
        e = {"launches": max(len(v) for v in d.values())}
        if "FETCH_SIZE" in d:
            e["fetch_bytes_raw"] = 1024.0 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
            e["fetch_bytes"] = 2.0 * e["fetch_bytes_raw"]      # gfx950 half-count correction
        if "WRITE_SIZE" in d:
            e["write_bytes"] = 1024.0 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        if "fetch_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
            if len(d["FETCH_SIZE"]) == len(d["WRITE_SIZE"]):
                # the largest launch (passes replay the same launch sequence)
                e["traffic_bytes_max"] = max(1024.0 * (2.0 * f + w)
                                             for f, w in zip(d["FETCH_SIZE"], d["WRITE_SIZE"]))
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU"):
            if c in d:
                e[c] = sum(d[c]) / len(d[c])
        res[k] = e
    json.dump({"source": "rocprofv3 --pmc, separate passes per counter group; FETCH_SIZE doubled "
                         "per MI355X_MICROARCH.md (gfx950 counts 64 B per 128 B request)",
               "kernels": res}, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
