"""Batched callers of the validity checker from MPlib's Python facade
(reference mplib/planner.py).

``generate_collision_pair`` is ``Planner.generate_collision_pair``
(planner.py:118-163) with its 10^6-iteration Python loop replaced by one
device call: the random full configurations (fingers included, as
``set_qpos(qpos, True)`` sets them) are drawn on the GPU, evaluated like
``collide_full()`` and counted per link pair on the device
(``PlanningWorld.sample_pair_counts``, C ABI ``mpg_collide_count``).  The
pairs that collide in every sample are written as ``disable_collisions``
entries of an SRDF, in the reference's format.

Sampling: each joint value is uniform in the joint's limits (pinocchio
``randomConfiguration``'s distribution; continuous joints over [-pi, pi]),
drawn by a counter-based generator (splitmix64 of seed and value index,
``sample_uniform`` below restates it) rather than ``std::rand``, so a batch
is reproducible and shardable; the statistic the SRDF rests on (a pair that
collides in every sample) does not depend on the stream.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from typing import List, Optional, Sequence, Tuple
from xml.dom import minidom

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def sample_uniform(lower: Sequence[float], upper: Sequence[float], n: int, seed: int, offset: int = 0) -> np.ndarray:
    """The device sampler (mpg_sample_uniform) on the host: value i of the
    batch (row-major, i = row * dof + k, counted from ``offset`` rows) is
    lower[k] + (upper[k] - lower[k]) * u, u = splitmix64(seed + (i + 1) *
    golden) >> 11 scaled by 2^-53."""
    lo = np.asarray(lower, np.float64)
    hi = np.asarray(upper, np.float64)
    dof = lo.size
    i = np.arange(offset * dof, (offset + n) * dof, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (lo + (hi - lo) * u.reshape(n, dof)).reshape(n, dof)


def collision_pair_counts(world, sample_time: int = 1000000, seed: int = 0) -> List[Tuple[str, str, int]]:
    """(link_name1, link_name2, count) per pair of the world's collide_full()
    table: in how many of ``sample_time`` random full configurations of the
    planned articulations the pair is reported."""
    counts = world.sample_pair_counts(int(sample_time), int(seed))
    info = world.get_collision_pair_info()
    return [(i[3], i[4], int(c)) for i, c in zip(info, counts)]


def generate_collision_pair(world, link_names: Sequence[str], urdf_path: str, sample_time: int = 1000000,
                            seed: int = 0, srdf_path: Optional[str] = None, verbose: bool = True) -> str:
    """Planner.generate_collision_pair (planner.py:118-163): count, per
    (link1, link2) of ``link_names`` (the planner's user links), the samples in
    which collide_full() reports the pair, and write every pair whose count is
    ``sample_time`` as ``<disable_collisions link1 link2 reason="Default"/>``
    to ``srdf_path`` (default: the URDF path with .srdf).  Returns the path."""
    idx = {n: i for i, n in enumerate(link_names)}
    cnt = np.zeros((len(link_names), len(link_names)), dtype=np.int64)
    for l1, l2, c in collision_pair_counts(world, sample_time, seed):
        if l1 in idx and l2 in idx:
            cnt[idx[l1]][idx[l2]] += c
    root = ET.Element("robot")
    root.set("name", urdf_path.split("/")[-1].split(".")[0])
    srdf = srdf_path or urdf_path.replace(".urdf", ".srdf")
    for i in range(len(link_names)):
        for j in range(len(link_names)):
            if cnt[i][j] == sample_time:
                if verbose:
                    print("Ignore collision pair: (%s, %s), reason:  always collide" % (link_names[i], link_names[j]))
                c = ET.SubElement(root, "disable_collisions")
                c.set("link1", link_names[i])
                c.set("link2", link_names[j])
                c.set("reason", "Default")
    with open(srdf, "w") as f:
        f.write(minidom.parseString(ET.tostring(root)).toprettyxml(indent="    "))
    if verbose:
        print("Saving the SRDF file to %s" % srdf)
    return srdf
