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
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Counter_Name"]][short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    res = {"configs_per_launch": n, "source": os.path.relpath(d), "hbm_bytes_per_launch": {}, "raw_kib": {}}
    stage = {"cull": "cull", "narrow": "narrow"}
    for k in set(vals["FETCH_SIZE"]) | set(vals["WRITE_SIZE"]):
        fk = vals["FETCH_SIZE"].get(k, [0.0])
        wk = vals["WRITE_SIZE"].get(k, [0.0])
        fetch = sum(fk) / len(fk) * 1024.0
        write = sum(wk) / len(wk) * 1024.0
        res["raw_kib"][k] = {"FETCH_SIZE": fetch / 1024.0, "WRITE_SIZE": write / 1024.0}
        res["hbm_bytes_per_launch"][stage.get(k, k)] = 2.0 * fetch + write
    for c in vals:
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            res.setdefault("other", {})[c] = {k: sum(v) / len(v) for k, v in vals[c].items()}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res["hbm_bytes_per_launch"]))


if __name__ == "__main__":
    main()
