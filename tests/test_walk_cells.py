"""Walk-hull direction tables (mpg_hullcells.h build_walk_cells): per
direction, the answer the device takes without climbing -- the trap-free
subcell's list maximum, or the trapped subcell's certified fine-cell endpoint
(walk_cone_endpoint), or the neighbour verification -- must be the vertex FCL
0.7.0's neighbour walk from vertex 0 ends at (oracle/collide_oracle.c
support_convex), replayed on the host by tests/native/walk_cells.cpp.  Also
bounds the share of directions left to the climb."""
import ctypes
import zlib

import numpy as np
import pytest

import worlds as Wd
from native.host_shim import walk_lib
from test_hullcells import adversarial_dirs


def _walk_hulls():
    ow = Wd.oracle_world(3)
    out = []
    for o in ow.art.objects:
        if len(o.geom.vertices) > 32:
            out.append((o.link, o.geom))
    return out


def check(geom, dirs, subk=8):
    V = np.ascontiguousarray(np.asarray(geom.vertices, np.float64).reshape(-1, 3))
    F = np.asarray([x for f in geom.faces for x in [len(f)] + list(f)], np.int32)
    d = np.ascontiguousarray(dirs, np.float64)
    st = np.zeros(12, np.int64)
    vp = ctypes.c_void_p
    r = walk_lib().walk_cells_check(V.ctypes.data_as(vp), len(V), F.ctypes.data_as(vp), len(geom.faces),
                                    d.ctypes.data_as(vp), ctypes.c_longlong(len(d)), subk, st.ctypes.data_as(vp))
    assert r == 0
    return st


@pytest.mark.parametrize("link,geom", _walk_hulls(), ids=[h[0] for h in _walk_hulls()])
def test_walk_tables_match_fcl_walk(link, geom):
    rng = np.random.default_rng(zlib.crc32(link.encode()))
    V = np.asarray(geom.vertices, np.float64).reshape(-1, 3)
    # MPR hands the support fp32 directions (libccd float build)
    d = np.vstack([rng.standard_normal((60000, 3)).astype(np.float32).astype(np.float64),
                   adversarial_dirs(V, rng, n_random=2000)[:40000]])
    st = check(geom, d)
    # (exact ties, cell boundaries and extreme magnitudes go to the climb)
    assert st[5] == 0, f"{st[5]} of {st[0]} directions disagree with the walk"
    assert st[1] + st[2] > 0.5 * st[0]


def test_walk_pending_share_small():
    rng = np.random.default_rng(5)
    tot = np.zeros(12, np.int64)
    for _, geom in _walk_hulls():
        tot += check(geom, rng.standard_normal((40000, 3)).astype(np.float32).astype(np.float64))
    assert tot[5] == 0
    assert tot[3] < 1e-3 * tot[0], tot  # certified fine cells settle the trapped subcells
    assert tot[6] < 0.15 * tot[7], tot  # most trapped fine cells have a certified endpoint


def test_cone_with_long_cell_lists():
    """a cone's base keeps ~300 rim vertices in one cell list; the
    record's count field must hold it (was n + 256 * offset)."""
    g = Wd.cone_hull(300)
    rng = np.random.default_rng(3)
    d = np.vstack([rng.standard_normal((20000, 3)), np.array([[0.0, 0.0, -1.0], [1e-3, 2e-3, -1.0]]),
                   rng.standard_normal((5000, 3)) * [0.05, 0.05, 1.0] - [0, 0, 2.0]])
    st = check(g, d.astype(np.float32).astype(np.float64))
    assert st[5] == 0, f"{st[5]} of {st[0]} directions disagree with the walk"
