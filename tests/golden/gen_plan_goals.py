#!/usr/bin/env python3
"""Offline generator of scenes.PLAN_GOALS: collision-free IK solutions of a
panda_hand pose in the cfg3 scene (least squares over the oracle's FK, random
restarts, first collision-free solution).  Test infrastructure only: the
product has no IK (out of scope)."""
import os
import sys

import numpy as np
from scipy.optimize import least_squares

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import worlds as Wd  # noqa: E402

ow = Wd.oracle_world(3)
lim = Wd.panda_articulation().joint_limits()[:7]
TQ = np.array([0.0, 1.0, 0.0, 0.0])


def ik(target):
    def f(q7):
        p = ow.fk_batch(q7[None])[0][0, 8]
        qq = p[3:] if np.dot(p[3:], TQ) >= 0 else -p[3:]
        return np.concatenate([p[:3] - target, 0.5 * (qq - TQ)])
    for s in range(40):
        rng = np.random.default_rng(s)
        q0 = np.array([0, 0.2, 0, -2.6, 0, 3.0, 0.8]) if s == 0 else rng.uniform(lim[:, 0], lim[:, 1])
        r = least_squares(f, q0, bounds=(lim[:, 0], lim[:, 1]), xtol=1e-15, ftol=1e-15, gtol=1e-15)
        if r.cost < 1e-20 and not ow.collide_batch(r.x[None])[0][0]:
            return np.round(r.x, 8)
    return None


if __name__ == "__main__":
    for tgt in [(0.4, 0.3, 0.2), (0.65, -0.15, 0.3)]:
        print(tgt, None if (g := ik(np.array(tgt))) is None else [float(v) for v in g])
