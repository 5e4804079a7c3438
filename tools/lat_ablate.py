"""Latency-path ablation: median round trip of collide_batch(N) for one
world; run under MPG_DEBUG_CULL=0/3/7 (full / no narrow test / FK only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
from latency import med  # noqa: E402
from mplib_amd import scenes  # noqa: E402

w, art = scenes.world(3)
for n in (1, 64, 128):
    q = scenes.sample_states(art, n, 3)
    print(os.environ.get("MPG_DEBUG_CULL", "0"), f"N={n}", round(med(lambda: w.collide_batch(q)), 1), "us", flush=True)
