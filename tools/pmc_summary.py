#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/profile.sh) into per-kernel HBM bytes
per launch, corrected as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
read, so reads are doubled.

usage: pmc_summary.py <profile_dir> <configs_per_launch> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"::(\w+?)(<|\()", name)
    return (m.group(1) if m else name).replace("_kernel", "")


def main():
    d, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)  # dispatch wall time of the pass that holds GRBM_GUI_ACTIVE (ns)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Counter_Name"]][short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
                dur[short(r["Kernel_Name"])].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from build_hash import build_hash
    res = {"configs_per_launch": n, "source": os.path.relpath(d),
           "lib_hash": build_hash(),
           "correction": "hbm_bytes = 2*FETCH_SIZE(KiB)*1024 + WRITE_SIZE(KiB)*1024 (MI355X_MICROARCH.md HBM section: "
                         "gfx950 FETCH_SIZE counts half of wide reads)",
           "kernels": defaultdict(dict)}
    for k in set(vals["FETCH_SIZE"]) | set(vals["WRITE_SIZE"]):
        fk = vals["FETCH_SIZE"].get(k, [0.0])
        wk = vals["WRITE_SIZE"].get(k, [0.0])
        fetch = sum(fk) / len(fk) * 1024.0
        write = sum(wk) / len(wk) * 1024.0
        res["kernels"][k].update({"FETCH_SIZE_KiB": fetch / 1024.0, "WRITE_SIZE_KiB": write / 1024.0,
                                  "hbm_bytes": 2.0 * fetch + write})
    for c in vals:  # per-launch averages of every other counter
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            for k, v in vals[c].items():
                res["kernels"][k][c] = sum(v) / len(v)
    # effective clock (MI355X_MICROARCH.md "DVFS give-back"): GRBM_GUI_ACTIVE is
    # summed over the 8 XCDs; divided by the dispatch's wall time in that pass
    for k, v in dur.items():
        ns = sum(v) / len(v)
        res["kernels"][k]["pmc_dispatch_ns"] = ns
        g = res["kernels"][k].get("GRBM_GUI_ACTIVE")
        if g and ns > 0:
            res["kernels"][k]["clock_ghz"] = g / 8.0 / ns
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v.get("hbm_bytes") for k, v in res["kernels"].items()}))


if __name__ == "__main__":
    main()
