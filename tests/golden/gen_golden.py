"""Generate tests/golden/* from the CPU oracle (oracle/).

The reference ships no golden vectors for this path, so
these fixtures are REGRESSION pins of the oracle restatement, not reference
outputs.  The only reference-sourced known answers are the two
examples/detect_collision.py configurations, stored in kat.json.

panda_mesh_1024 (BVH-mesh Panda) was regenerated in round 4 when the oracle
began restating FCL's OBBRSS traversal: one bit, masks[892] pair 47
(panda_link6 - green_cube), flipped from hit to miss -- float MPR reports a
false hit 1.75 mm off the surface, and FCL's OBB test on the path to that
triangle's leaf fails, so FCL never runs that leaf.  The fixture therefore
pins the device to the oracle's restatement of that traversal; FCL itself is
not importable here, so the bit's parity with FCL is unpinned.
Run:  python tests/golden/gen_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import worlds as Wd  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
os.makedirs(OUT, exist_ok=True)


def vectors(cfg, n, name):
    ow = Wd.oracle_world(cfg)
    q = Wd.sample_q(ow.art, n, Wd.CFG_SEED[cfg])
    fl, mk = ow.collide_batch(q, nthreads=8)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), q=q, flags=fl, masks=mk,
                        pairs=np.array([list(p) for p in ow.pair_names()]))
    print(name, "collision rate", fl.mean())


def main():
    if "--only" in sys.argv:  # one fixture, e.g. --only 7 panda_mesh_1024
        k = sys.argv.index("--only")
        vectors(int(sys.argv[k + 1]), 1024, sys.argv[k + 2])
        return
    ow2 = Wd.oracle_world(2)
    art = ow2.art
    # model facts + pair table
    facts = {
        "objects": [o.link for o in art.objects],
        "vertex_counts": [int(len(o.geom.vertices)) for o in art.objects],
        "self_pairs": [[int(a), int(b)] for a, b in art.pairs],
        "self_pair_names": [[art.objects[a].link, art.objects[b].link] for a, b in art.pairs],
        "joint_types": [art.pin.joint_type_name(j) for j in range(1, len(art.pin.joints))],
        "link0_min_z": float(art.objects[0].geom.vertices[:, 2].min()),
    }
    with open(os.path.join(OUT, "panda_model.json"), "w") as fh:
        json.dump(facts, fh, indent=1)
    # known answers from examples/detect_collision.py:25,31
    f, m = ow2.collide_batch(np.array([Wd.KAT_FREE, Wd.KAT_COLLIDING]))
    kat = {"free": {"q": Wd.KAT_FREE, "collides": bool(f[0]), "pairs": ow2.decode(m[0])},
           "colliding": {"q": Wd.KAT_COLLIDING, "collides": bool(f[1]), "pairs": ow2.decode(m[1])}}
    with open(os.path.join(OUT, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    # per-config vectors
    for cfg, n, name in [(2, 4096, "panda_self_4096"), (3, 4096, "panda_boxes_4096"), (4, 1024, "panda_convex_1024"),
                         (7, 1024, "panda_mesh_1024")]:
        vectors(cfg, n, name)
    q = Wd.sample_q(art, 64, 7)
    poses, objT = ow2.fk_batch(q)
    np.savez_compressed(os.path.join(OUT, "panda_fk_64.npz"), q=q, link_pose=poses, obj_T=objT)


if __name__ == "__main__":
    main()
