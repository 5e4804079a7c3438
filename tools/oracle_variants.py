#!/usr/bin/env python3
"""Oracle-variant study (DESIGN.md "Oracle variants").

The oracle restates FCL 0.7.0 / libccd 2.1 / pinocchio 2.6.21 / Eigen 3.4.0
arithmetic that is not present in this image.  A few restatement choices could
not be pinned from the reference's files alone; each is compiled as a variant
of oracle/collide_oracle.c (oracle.VARIANTS) and run on the BASELINE batches.
This script counts, per variant, the configurations whose collide() flag and
the (configuration, pair) bits whose collideFull() report differ from the
default oracle, and the FK link-pose bits that differ.

usage: python tools/oracle_variants.py [--threads 8] [--cfgs 2,3,4] [--n4 262144] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402  (test infrastructure: this is a checker study)
import worlds as Wd  # noqa: E402


def popcount(a: np.ndarray) -> int:
    return int(np.unpackbits(a.view(np.uint8)).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--cfgs", default="2,3,4")
    ap.add_argument("--n4", type=int, default=1 << 18, help="cfg4 sample size (BASELINE: 2^22)")
    ap.add_argument("--variants", default=",".join(oracle.VARIANTS))
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    out = {"threads": args.threads, "rows": []}
    for cfg in [int(c) for c in args.cfgs.split(",")]:
        ow = Wd.oracle_world(cfg)
        n = Wd.CFG_N[cfg] if cfg != 4 else args.n4
        q = Wd.sample_q(ow.art, n, Wd.CFG_SEED[cfg])
        t0 = time.perf_counter()
        f0, m0 = ow.collide_batch(q, nthreads=args.threads)
        dt0 = time.perf_counter() - t0
        p0, _ = ow.fk_batch(q[: 1 << 14])
        base = {"cfg": cfg, "n": n, "variant": "default", "hits": int(f0.sum()), "pair_bits": popcount(m0),
                "seconds": dt0}
        print(json.dumps(base), flush=True)
        out["rows"].append(base)
        for v in args.variants.split(","):
            t0 = time.perf_counter()
            f1, m1 = ow.collide_batch(q, nthreads=args.threads, variant=v)
            dt = time.perf_counter() - t0
            lib = oracle.variant_lib(v)
            poses = np.zeros_like(p0)
            qq = np.ascontiguousarray(q[: 1 << 14])
            lib.orc_fk_batch(oracle.ctypes.byref(ow._w), qq.ctypes.data_as(oracle._DP), oracle.ctypes.c_long(len(qq)),
                             poses.ctypes.data_as(oracle._DP), None)
            diff_cfg = np.nonzero(f0 != f1)[0]
            xm = m0 ^ m1
            row = {"cfg": cfg, "n": n, "variant": v, "flag_diffs": int(len(diff_cfg)),
                   "flags_set_by_variant_only": int(((f1 == 1) & (f0 == 0)).sum()),
                   "flags_cleared_by_variant": int(((f1 == 0) & (f0 == 1)).sum()),
                   "pair_bit_diffs": popcount(xm),
                   "configs_with_pair_diffs": int((xm != 0).any(axis=1).sum()),
                   "fk_pose_values_differing": int((poses != p0).sum()),
                   "fk_max_abs_diff": float(np.abs(poses - p0).max()),
                   "first_diff_configs": diff_cfg[:5].tolist(),
                   "seconds": dt}
            print(json.dumps(row), flush=True)
            out["rows"].append(row)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
