"""C18 oracle pinning (CPU): the generated marching-cubes case table (oracle vs the library's
independent constexpr generator, read through the host-only ldm_mc_table), and mesh
properties that pin the algorithm without a reference library (none is installed, SURVEY.md
P3): closed, consistently oriented 2-manifolds with the right Euler characteristic, outward
normals, vertices on the analytic surface, single-cube known answers, PLY round trip."""
from collections import defaultdict

import numpy as np
import pytest

from oracle import ref_mc as M


def _mesh_stats(v, f):
    D = defaultdict(int)
    for a, b, c in f:
        for p, q in ((a, b), (b, c), (c, a)):
            D[(p, q)] += 1
    und = {(min(p, q), max(p, q)) for p, q in D}
    dup = sum(1 for n in D.values() if n > 1)
    unpaired = sum(1 for (p, q) in D if (q, p) not in D)
    return dup, unpaired, len(v) - len(und) + len(f)


def _grid(N):
    c = M._coords(N)
    return np.meshgrid(c, c, c, indexing="ij")          # z, y, x


def test_library_table_equals_oracle_table():
    import ldm_sdf
    tri, ntri = ldm_sdf.mc_table()
    tri_o, ntri_o = M.mc_tables()
    assert np.array_equal(tri, tri_o) and np.array_equal(ntri, ntri_o)


def test_table_shape_properties():
    tri, ntri = M.mc_tables()
    assert ntri[0] == 0 and ntri[255] == 0 and ntri.max() == 5
    for cfg in range(256):
        used = tri[cfg, :3 * ntri[cfg]]
        assert (used >= 0).all() and (used < 12).all() and (tri[cfg, 3 * ntri[cfg]:] == -1).all()
        # the edges a case uses are exactly its sign-changing edges
        crossing = set()
        for e in range(12):
            c0, c1 = M.edge_corners(e)
            if ((cfg >> c0) & 1) != ((cfg >> c1) & 1):
                crossing.add(e)
        assert set(used.tolist()) == crossing, cfg


def test_single_corner_known_answer():
    """Only corner 0 inside: one triangle on the 3 edges from it, at the exact fp32
    interpolation points, normal pointing away from the corner."""
    vol = np.ones((2, 2, 2), np.float32)
    vol[0, 0, 0] = -1.0 / 3.0                                 # t = 0.25 on every edge
    v, f = M.marching_cubes(vol, 0.0, bbox=(0.0, 1.0))
    assert f.shape == (1, 3) and v.shape == (3, 3)
    want = {(0.25, 0.0, 0.0), (0.0, 0.25, 0.0), (0.0, 0.0, 0.25)}
    assert {tuple(map(float, p)) for p in v} == want
    n = np.cross(v[f[0, 1]] - v[f[0, 0]], v[f[0, 2]] - v[f[0, 0]])
    assert np.all(n > 0)


def test_sphere_closed_outward_on_surface():
    z, y, x = _grid(48)
    r = np.sqrt(x * x + y * y + z * z)
    v, f = M.marching_cubes((r - 0.6).astype(np.float32))
    dup, unpaired, chi = _mesh_stats(v, f)
    assert dup == 0 and unpaired == 0 and chi == 2
    cen = v[f].mean(1)
    nrm = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    assert np.all((nrm * cen).sum(1) > 0)
    h = 2.0 / 47
    assert np.abs(np.linalg.norm(v, axis=1) - 0.6).max() < 0.1 * h


def test_plane_vertices_exact():
    """A linear field: every vertex lies on the plane up to fp32 rounding of the interpolation."""
    z, y, x = _grid(20)
    vol = (0.3 * x - 0.5 * y + 0.81 * z - 0.05).astype(np.float32)
    v, f = M.marching_cubes(vol)
    res = 0.3 * v[:, 0] - 0.5 * v[:, 1] + 0.81 * v[:, 2] - 0.05
    assert len(f) > 0 and np.abs(res).max() < 1e-5


def test_torus_genus_one():
    z, y, x = _grid(48)
    tor = np.sqrt((np.sqrt(x * x + y * y) - 0.5) ** 2 + z * z) - 0.2
    v, f = M.marching_cubes(tor.astype(np.float32))
    dup, unpaired, chi = _mesh_stats(v, f)
    assert dup == 0 and unpaired == 0 and chi == 0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_closed_volumes_are_oriented_manifolds(seed):
    """Every ambiguous face / cube configuration shows up in white noise; padding with a
    positive border closes the surface, so every edge must pair with its reverse."""
    rng = np.random.default_rng(seed)
    n = 14
    vol = np.ones((n + 2,) * 3, np.float32)
    vol[1:-1, 1:-1, 1:-1] = rng.standard_normal((n, n, n))
    v, f = M.marching_cubes(vol)
    dup, unpaired, chi = _mesh_stats(v, f)
    assert dup == 0 and unpaired == 0 and chi % 2 == 0
    nb = defaultdict(dict)                                   # vertex links are single cycles
    for a, b, c in f:
        nb[a][b] = c
        nb[b][c] = a
        nb[c][a] = b
    for vert, ring in nb.items():
        s = next(iter(ring))
        cur, cnt = s, 0
        while True:
            cur = ring[cur]
            cnt += 1
            if cur == s:
                break
        assert cnt == len(ring), vert


def test_empty_and_level():
    vol = np.ones((5, 5, 5), np.float32)
    v, f = M.marching_cubes(vol)
    assert v.shape == (0, 3) and f.shape == (0, 3)
    v2, f2 = M.marching_cubes(vol, level=2.0)                # everything inside: no surface
    assert len(f2) == 0


def test_ply_round_trip(tmp_path):
    import ldm_sdf
    z, y, x = _grid(16)
    v, f = M.marching_cubes((np.sqrt(x * x + y * y + z * z) - 0.5).astype(np.float32))
    p = str(tmp_path / "m.ply")
    ldm_sdf.write_ply(p, v, f)
    v2, f2 = M.read_ply(p)
    assert np.array_equal(v, v2) and np.array_equal(f, f2)
    with open(p, "rb") as fh:
        assert fh.read(60).startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex")
