"""Direction-cell candidate lists of the Convex support (mpg_hullcells.h):
the support through a cell's list must equal the full first-maximum scan
(oracle/collide_oracle.c support_convex) for every direction, including
facet normals (exact ties), cell-boundary directions, duplicated and
non-extreme vertices and extreme magnitudes."""
import ctypes
import zlib

import numpy as np
import pytest

import worlds as Wd
from native.host_shim import lib

K = 16  # mpg_hullcells.h kCellK


def support_pair(V, dirs):
    V = np.ascontiguousarray(V, dtype=np.float64)
    dirs = np.ascontiguousarray(dirs, dtype=np.float64)
    n = len(dirs)
    full = np.zeros((n, 3))
    cell = np.zeros((n, 3))
    stats = np.zeros(3, dtype=np.int64)
    P = ctypes.POINTER(ctypes.c_double)
    f = lib().host_hull_support
    f.restype = ctypes.c_long
    bad = f(V.ctypes.data_as(P), ctypes.c_int(len(V)), dirs.ctypes.data_as(P), ctypes.c_long(n),
            full.ctypes.data_as(P), cell.ctypes.data_as(P), stats.ctypes.data_as(ctypes.POINTER(ctypes.c_long)))
    return bad, full, cell, stats


def adversarial_dirs(V, rng, n_random=20000):
    d = [rng.standard_normal((n_random, 3))]
    # hull facet normals and vertex/edge directions: exact and near ties
    try:
        from scipy.spatial import ConvexHull
        h = ConvexHull(V)
        nrm = h.equations[:, :3]
        d += [nrm, -nrm, nrm + 1e-12 * rng.standard_normal(nrm.shape)]
        e = V[h.simplices[:, 0]] - V[h.simplices[:, 1]]
        d += [np.cross(e, nrm)]
    except Exception:
        pass
    d += [V - V.mean(0), V[rng.integers(0, len(V), 500)] - V[rng.integers(0, len(V), 500)]]
    # cell boundaries and cube-face boundaries, exact and 1 ulp off
    b = -1.0 + 2.0 * np.arange(K + 1) / K
    u, v = np.meshgrid(b, rng.uniform(-1, 1, 8))
    u, v = u.ravel(), v.ravel()
    for sgn in (1.0, -1.0):
        for f in range(3):
            for uu in (u, np.nextafter(u, 2), np.nextafter(u, -2)):
                x = np.zeros((len(u), 3))
                x[:, f] = sgn
                x[:, (f + 1) % 3] = uu
                x[:, (f + 2) % 3] = v
                d += [x, x[:, [0, 2, 1]]]
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], float)
    axes = np.vstack([np.eye(3), -np.eye(3), [[1, 1, 0], [0, -1, 1], [1, 0, -1], [-0.0, 0.0, 1.0]]])
    d += [corners, axes, np.nextafter(corners, 0)]
    D = np.vstack(d)
    # magnitudes: unit scale, small and large (cells), extreme (full-scan path)
    scales = [1.0, 1e-25, 1e25, 1e-40, 1e40]
    out = [D * s for s in scales]
    out.append(np.array([[0.0, 0.0, 0.0], [np.nan, 1.0, 0.0], [1.0, np.inf, 0.0], [-np.inf, 0.0, 0.0],
                         [0.0, np.nan, np.nan], [1.0, 1.0, np.nan]]))
    return np.vstack(out)


def hulls():
    ow = Wd.oracle_world(3)
    out = [("panda_" + str(i), np.asarray(o.geom.vertices).reshape(-1, 3)) for i, o in enumerate(ow.art.objects)]
    rng = np.random.default_rng(7)
    cube = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], float) * 0.05
    out.append(("cube", cube))
    # duplicated vertices and non-extreme points on the faces and inside
    g = np.linspace(-0.05, 0.05, 5)
    face = np.array([[x, y, 0.05] for x in g for y in g])
    out.append(("cube_dup_face", np.vstack([cube, cube[::-1], face, 0.01 * rng.standard_normal((20, 3))])))
    s = rng.standard_normal((300, 3))
    out.append(("sphere300", 0.1 * s / np.linalg.norm(s, axis=1, keepdims=True)))
    out.append(("tiny", 1e-4 * rng.standard_normal((40, 3))))
    out.append(("large", 1e3 * rng.standard_normal((40, 3))))
    out.append(("offset", rng.standard_normal((60, 3)) * 0.02 + np.array([3.0, -2.0, 1.0])))
    out.append(("flat", np.c_[rng.standard_normal((50, 2)), np.zeros(50)]))
    out.append(("single", np.array([[0.1, 0.2, 0.3]])))
    return out


@pytest.mark.parametrize("name,V", hulls(), ids=[h[0] for h in hulls()])
def test_cell_support_equals_full_scan(name, V):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    dirs = adversarial_dirs(V, rng)
    bad, full, cell, stats = support_pair(V, dirs)
    assert bad == 0, f"{bad} of {len(dirs)} directions differ"
    np.testing.assert_array_equal(full, cell)
    assert stats[0] > 0.55 * len(dirs)  # all but the extreme-magnitude directions use a cell


def test_panda_lists_are_short():
    # the point of the lists: a few candidates per cell instead of ~120 vertices
    ow = Wd.oracle_world(3)
    rng = np.random.default_rng(3)
    dirs = rng.standard_normal((20000, 3))
    for o in ow.art.objects:
        V = np.asarray(o.geom.vertices).reshape(-1, 3)
        bad, _, _, stats = support_pair(V, dirs)
        assert bad == 0
        assert stats[1] / stats[0] < 4.0, (len(V), stats)
