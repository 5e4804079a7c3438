"""The BASELINE.json benchmark worlds, built through the product API
(``mplib_amd.pymp``) exactly as a user of the reference would build them.

  cfg2  Panda self-collision (2^16 states, default_rng(0))
  cfg3  Panda + 10 boxes: collision_avoidance.py:29-59 table/red/green/blue
        (side = 2 x half_size) + 6 boxes from default_rng(1234);
        ACM (panda_link0, table) = ALWAYS  (2^20 states, default_rng(1))
  cfg4  Panda + 4 convex hulls (link3/link5/hand/link0 hulls at poses from
        default_rng(4321))  (2^22 states sharded over GPUs, default_rng(2))
  cfg5  RRTConnect plan() in the cfg3 scene (PLAN_START -> PLAN_GOALS)
  cfg6  Panda + the detect_collision.py floor point cloud (fcl::OcTree,
        10000 points, resolution 1e-3)  (2^20 states, default_rng(6))

States are uniform in the URDF joint limits (panda.urdf:37-157).
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np

from . import pymp

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PANDA_DIR = os.path.join(_ROOT, "data", "panda")
PANDA_LINKS = ["panda_link0", "panda_link1", "panda_link2", "panda_link3", "panda_link4", "panda_link5",
               "panda_link6", "panda_link7", "panda_hand", "panda_leftfinger", "panda_rightfinger"]
PANDA_JOINTS = ["panda_joint1", "panda_joint2", "panda_joint3", "panda_joint4", "panda_joint5", "panda_joint6",
                "panda_joint7", "panda_finger_joint1", "panda_finger_joint2"]
CFG_SEED = {2: 0, 3: 1, 4: 2, 6: 6, 7: 7}
CFG_N = {2: 1 << 16, 3: 1 << 20, 4: 1 << 22, 6: 1 << 20, 7: 1 << 18}
CFG_NAME = {2: "panda_self", 3: "panda_10boxes", 4: "panda_4convex", 6: "panda_floor_cloud",
            7: "panda_bvh_meshes_10boxes"}


def panda(convex: bool = True) -> "pymp.articulation.ArticulatedModel":
    """convex=False loads the collision meshes as BVH triangle meshes
    (load_mesh_as_BVH, fcl_model.cpp:224-227)."""
    a = pymp.articulation.ArticulatedModel(os.path.join(PANDA_DIR, "panda.urdf"), os.path.join(PANDA_DIR, "panda.srdf"),
                                           [0, 0, -9.81], PANDA_JOINTS, PANDA_LINKS, verbose=False, convex=convex)
    a.set_move_group("panda_hand")
    return a


def _boxes():
    out = [("table", (0.8, 0.8, 0.05), (0.56, 0.0, -0.025)),
           ("red_cube", (0.04, 0.04, 0.12), (0.7, 0.0, 0.06)),
           ("green_cube", (0.08, 0.08, 0.01), (0.4, 0.3, 0.005)),
           ("blue_cube", (0.1, 0.4, 0.2), (0.55, 0.0, 0.1))]
    rng = np.random.default_rng(1234)
    for k in range(6):
        side = rng.uniform(0.02, 0.2, size=3)
        c = rng.uniform([0.2, -0.5, 0.05], [0.8, 0.5, 0.8])
        out.append((f"box{k}", tuple(float(s) for s in side), tuple(float(v) for v in c)))
    return out


def _hulls():
    rng = np.random.default_rng(4321)
    out = []
    for k, name in enumerate(["link3", "link5", "hand", "link0"]):
        pos = rng.uniform([0.3, -0.5, 0.0], [0.8, 0.5, 0.7])
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        out.append((f"hull{k}_panda_{name}", name, [float(v) for v in pos], [float(v) for v in q]))
    return out


def world(cfg: int, convex: bool = True):
    """(PlanningWorld, ArticulatedModel) for a BASELINE config (6: the
    detect_collision.py floor point cloud, see cloud_world); convex=False:
    the robot's links as BVH meshes."""
    if cfg == 6:
        return cloud_world("floor")
    if cfg == 7:  # cfg3 with the links as BVH meshes (convex=False)
        return world(3, convex=False)
    art = panda(convex)
    w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
    if cfg == 3:
        for name, side, pos in _boxes():
            w.add_normal_object(name, pymp.fcl.CollisionObject(pymp.fcl.Box(list(side)), list(pos), [1, 0, 0, 0]))
        w.get_allowed_collision_matrix().set_entry("panda_link0", "table", True)
    elif cfg == 4:
        mesh_dir = os.path.join(PANDA_DIR, "franka_description", "meshes", "collision")
        for name, mesh, pos, quat in _hulls():
            g = pymp.fcl.load_mesh_as_Convex(os.path.join(mesh_dir, mesh + ".stl.convex.stl"), [1, 1, 1])
            w.add_normal_object(name, pymp.fcl.CollisionObject(g, pos, quat))
    elif cfg != 2:
        raise ValueError(f"unknown config {cfg}")
    return w, art


def joint_limits(art) -> np.ndarray:
    lims = art.get_pinocchio_model().get_joint_limits()
    return np.array([l[0] for l in lims[:7]], dtype=np.float64)


def sample_states(art, n: int, seed: int) -> np.ndarray:
    lim = joint_limits(art)
    return np.random.default_rng(seed).uniform(lim[:, 0], lim[:, 1], size=(n, 7))


# cfg5 (BASELINE.json configs[4]): RRTConnect plan() in the cfg3 scene.
# Start: tests/test_basic.py:44 qpos (it touches the synthetic box1 in this
# scene, so plan() resamples it nearby as ompl_planner.cpp:110-115 does).
# Goals: collision-free IK solutions for the panda_hand pose (x, y, z, w=0,
# x=1, y=0, z=0) -- test_basic.py:43's pose (0.4, 0.3, 0.12) grips into the
# green cube here, so "near" is 8 cm above it; "far" reaches around box0 /
# box1 / box2 (a few hundred RRTConnect iterations).  Computed offline by
# least squares on the FK (tests/golden/gen_plan_goals.py), rounded to 1e-8.
PLAN_START = [0.0, 0.2, 0.0, -2.6, 0.0, 3.0, 0.8]
PLAN_GOALS = {
    "near": [0.33129616, 0.29436923, 0.29083465, -2.39517156, -0.1845193, 2.67095513, 1.56051207],  # (0.4, 0.3, 0.2)
    "far": [-2.41007622, -1.08236711, 1.81200205, -1.64528436, 1.08547798, 1.8186026, -0.00635181],  # (0.65, -0.15, 0.3)
}


# Point-cloud worlds (PlanningWorld.add_point_cloud -> fcl::OcTree), the
# reference examples' clouds with a numpy sampler in place of trimesh's
# sample_surface (uniform on the box faces, area weighted):
#   "floor": detect_collision.py:37-46 -- 10000 points on a 2 x 2 x 0.1 box
#            shifted down 0.1 (default_rng(8)), resolution 1e-3
#   "blue":  collision_avoidance.py:61-67 -- 1000 points on the blue cube's
#            surface (0.1 x 0.4 x 0.2 at (0.55, 0, 0.1), default_rng(7)), in
#            the cfg3 box scene, resolution 1e-3
def box_surface_points(rng, side, n: int, center) -> np.ndarray:
    side = np.asarray(side, dtype=np.float64)
    areas = np.array([side[1] * side[2], side[0] * side[2], side[0] * side[1]])
    face = rng.choice(3, n, p=areas / areas.sum())
    sgn = rng.choice([-1.0, 1.0], n)
    pts = rng.uniform(-side / 2, side / 2, (n, 3))
    pts[np.arange(n), face] = sgn * side[face] / 2
    return pts + np.asarray(center, dtype=np.float64)


def cloud_points(kind: str) -> np.ndarray:
    if kind == "floor":
        return box_surface_points(np.random.default_rng(8), (2.0, 2.0, 0.1), 10000, (0.0, 0.0, -0.1))
    if kind == "blue":
        return box_surface_points(np.random.default_rng(7), (0.1, 0.4, 0.2), 1000, (0.55, 0.0, 0.1))
    raise ValueError(kind)


def cloud_world(kind: str, resolution: float = 1e-3):
    """(PlanningWorld, ArticulatedModel) with the point cloud `kind` as 'scene_pcd'."""
    if kind == "floor":
        art = panda()
        w = pymp.planning_world.PlanningWorld([art], ["panda"], [], [])
    else:
        w, art = world(3)
    w.add_point_cloud("scene_pcd", cloud_points(kind), resolution)
    return w, art


# detect_collision.py:47-55: "this pose causes several joints to dip below the floor"
FLOOR_COLLIDING = [0.0, 1.5, 0.0, -1.5, 0.0, 0.0, 0.0]
