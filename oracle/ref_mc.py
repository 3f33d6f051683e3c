"""CPU oracle for marching cubes + PLY export.  TEST
INFRASTRUCTURE ONLY -- imported by ``tests/`` (and ``bench.py``'s cpu_baseline leg), never by
the product (``ldm_sdf.marching_cubes`` runs ``ldm_mc_*`` in HIP).

PARITY STATUS: unpinned by the reference (``/root/reference`` is ``README.md:1`` only), and no
marching-cubes library (skimage, mcubes, trimesh) is installed here.  The
algorithm is build-defined in DESIGN.md §10 -- Lorensen & Cline marching cubes with a fixed,
face-local ambiguity rule -- and its case table is GENERATED from that rule (below), not
transcribed.  The product generates its table independently (``csrc/mc.hip``, constexpr C++);
``tests/test_mc_oracle.py`` pins both: identical tables, watertight and consistently oriented
meshes on random volumes, Euler characteristics of spheres (2) and tori (0), and vertex
positions on the analytic surface.

Conventions (shared with the product):
* Volume ``[N, N, N]`` indexed ``[k][j][i]`` (z slowest, x fastest); grid coordinates by A1.
* Corner c of a cube has offset (c & 1, (c >> 1) & 1, (c >> 2) & 1) in (x, y, z); a corner is
  *inside* when ``v < level`` (strict).
* Cube edge ``e = 4 a + m`` runs along axis ``a`` from the corner whose other two bits (lower
  axis first) are ``m``; its vertex is owned by that start corner's grid point.
* A crossing edge gets ONE vertex (shared by the up-to-4 cubes around it): vertices are
  numbered by owner point (linear index) then axis; position
  ``p0 + t (p1 - p0)`` with ``t = (level - v0) / (v1 - v0)``, every op rounded to fp32.
* Faces: per cube in linear order, the case table's triangles in order; the winding makes
  ``(b - a) x (c - a)`` point toward increasing values (outside).
"""
from __future__ import annotations

import struct
from typing import List, Tuple

import numpy as np

__all__ = ["mc_tables", "marching_cubes", "write_ply", "read_ply"]


def _corner(a_bit_axis: int, s: int, ub: int, u: int, wb: int, w: int) -> int:
    return (s << a_bit_axis) | (ub << u) | (wb << w)


def _edge_id(c0: int, c1: int) -> int:
    d = c0 ^ c1
    a = {1: 0, 2: 1, 4: 2}[d]
    others = [b for b in range(3) if b != a]           # lower axis first
    lo = c0 & c1
    m = ((lo >> others[0]) & 1) | (((lo >> others[1]) & 1) << 1)
    return 4 * a + m


def edge_corners(e: int) -> Tuple[int, int]:
    a, m = divmod(e, 4)
    others = [b for b in range(3) if b != a]
    c0 = ((m & 1) << others[0]) | (((m >> 1) & 1) << others[1])
    return c0, c0 | (1 << a)


def _faces() -> List[List[int]]:
    """The 6 faces as corner lists in counter-clockwise order seen from outside the cube."""
    faces = []
    for a in range(3):
        u, w = (a + 1) % 3, (a + 2) % 3
        for s in (0, 1):
            ring = [(0, 0), (1, 0), (1, 1), (0, 1)]           # CCW about +e_a in (u, w)
            if s == 0:
                ring = ring[::-1]                              # outward normal is -e_a
            faces.append([_corner(a, s, ub, u, wb, w) for ub, wb in ring])
    return faces


def _edge_faces(e: int, faces: List[List[int]]) -> List[int]:
    c0, c1 = edge_corners(e)
    return [fi for fi, f in enumerate(faces) if c0 in f and c1 in f]


def _fan_start(cyc: List[int], faces: List[List[int]]) -> List[int]:
    """Rotate a polygon so that no fan diagonal from its first vertex lies in a cube face
    (two non-adjacent vertices on one face): such a diagonal would coincide with the
    neighbouring cube's geometry and break the manifold.  First valid rotation wins."""
    n = len(cyc)
    for r in range(n):
        rot = cyc[r:] + cyc[:r]
        f0 = set(_edge_faces(rot[0], faces))
        if all(not (f0 & set(_edge_faces(rot[i], faces))) for i in range(2, n - 1)):
            return rot
    raise AssertionError(f"no face-free fan for polygon {cyc}")


def mc_tables() -> Tuple[np.ndarray, np.ndarray]:
    """Generate (tri [256, 16] int8 edge ids, -1 padded; ntri [256] uint8).

    Face rule: walking a face's corners counter-clockwise from outside, each crossing where
    the walk leaves the inside connects to the closest crossing BEFORE it where the walk
    enters the inside (so two diagonal inside corners are cut off separately).  This gives,
    per crossing edge, exactly one successor; the successor cycles (listed from their
    smallest edge id) are the polygons, fanned from the first vertex whose fan diagonals
    avoid the cube faces.  Fan order (v0, v_{i+1}, v_i) orients normals outward.
    """
    faces = _faces()
    tri = -np.ones((256, 16), np.int8)
    ntri = np.zeros(256, np.uint8)
    for cfg in range(256):
        inside = [(cfg >> c) & 1 for c in range(8)]
        nxt = {}
        for f in faces:
            cross = []                                         # (edge, 'out' | 'in') in CCW order
            for q in range(4):
                A, B = f[q], f[(q + 1) % 4]
                if inside[A] != inside[B]:
                    cross.append((_edge_id(A, B), "out" if inside[A] else "in"))
            for q, (e, kind) in enumerate(cross):
                if kind != "out":
                    continue
                r = (q - 1) % len(cross)
                while cross[r][1] != "in":
                    r = (r - 1) % len(cross)
                nxt[e] = cross[r][0]
        tris: List[int] = []
        seen = set()
        for start in sorted(nxt):
            if start in seen:
                continue
            cyc = [start]
            seen.add(start)
            e = nxt[start]
            while e != start:
                cyc.append(e)
                seen.add(e)
                e = nxt[e]
            cyc = _fan_start(cyc, faces)
            for i in range(1, len(cyc) - 1):
                tris += [cyc[0], cyc[i + 1], cyc[i]]
        ntri[cfg] = len(tris) // 3
        tri[cfg, :len(tris)] = tris
    return tri, ntri


def _coords(N: int, bbox=(-1.0, 1.0)) -> np.ndarray:
    lo, hi = bbox
    vs = np.float32((hi - lo) / (N - 1))
    return ((np.arange(N, dtype=np.float32) * vs).astype(np.float32) + np.float32(lo)).astype(np.float32)


def marching_cubes(vol: np.ndarray, level: float = 0.0, bbox=(-1.0, 1.0)):
    """(verts float32 [V, 3] (x, y, z), faces int32 [F, 3]) -- DESIGN.md §10 conventions."""
    vol = np.asarray(vol, np.float32)
    N = vol.shape[0]
    assert vol.shape == (N, N, N) and N >= 2
    lv = np.float32(level)
    tri, ntri = mc_tables()
    ins = vol < lv                                             # [k][j][i]
    # ---- vertices: owner point (linear index) then axis x, y, z
    cross = np.zeros((N, N, N, 3), bool)
    cross[:, :, :-1, 0] = ins[:, :, :-1] != ins[:, :, 1:]
    cross[:, :-1, :, 1] = ins[:, :-1, :] != ins[:, 1:, :]
    cross[:-1, :, :, 2] = ins[:-1, :, :] != ins[1:, :, :]
    flat = cross.reshape(-1, 3)
    idx = np.flatnonzero(flat.reshape(-1))                     # (point * 3 + axis), sorted
    pt, ax = idx // 3, idx % 3
    k, j, i = pt // (N * N), (pt // N) % N, pt % N
    vofs = np.full(N * N * N * 3, -1, np.int64)
    vofs[idx] = np.arange(idx.size)
    c = _coords(N, bbox)
    di = (ax == 0).astype(np.int64)
    dj = (ax == 1).astype(np.int64)
    dk = (ax == 2).astype(np.int64)
    v0 = vol[k, j, i]
    v1 = vol[k + dk, j + dj, i + di]
    t = ((lv - v0).astype(np.float32) / (v1 - v0).astype(np.float32)).astype(np.float32)
    p0 = np.stack([c[i], c[j], c[k]], 1)
    p1 = np.stack([c[i + di], c[j + dj], c[k + dk]], 1)
    verts = (p0 + (t[:, None] * (p1 - p0).astype(np.float32)).astype(np.float32)).astype(np.float32)
    # ---- faces: cubes in linear order (min-corner point index), table order
    cfg = np.zeros((N - 1, N - 1, N - 1), np.int64)
    for cc in range(8):
        dx, dy, dz = cc & 1, (cc >> 1) & 1, (cc >> 2) & 1
        cfg |= ins[dz:N - 1 + dz, dy:N - 1 + dy, dx:N - 1 + dx].astype(np.int64) << cc
    ck, cj, ci = np.nonzero(ntri[cfg] > 0)                     # C order == linear cube order
    cfgs = cfg[ck, cj, ci]
    faces = []
    nt = ntri[cfgs].astype(np.int64)
    rep = np.repeat(np.arange(cfgs.size), nt)
    slot = np.arange(rep.size) - np.repeat(np.cumsum(nt) - nt, nt)
    ev = tri[cfgs[rep]][np.arange(rep.size)[:, None], 3 * slot[:, None] + np.arange(3)[None, :]]
    a = ev // 4
    m = ev % 4
    # start corner of each edge (DESIGN.md §10 edge numbering)
    sx = np.where(a == 0, 0, m & 1)
    sy = np.where(a == 0, m & 1, np.where(a == 1, 0, (m >> 1) & 1))
    sz = np.where(a == 2, 0, (m >> 1) & 1)
    owner = ((ck[rep][:, None] + sz) * N + (cj[rep][:, None] + sy)) * N + (ci[rep][:, None] + sx)
    faces = vofs[owner * 3 + a]
    assert (faces >= 0).all()
    return verts, faces.astype(np.int32)


def write_ply(path: str, verts: np.ndarray, faces: np.ndarray) -> None:
    """Binary little-endian PLY as DeepSDF's ``convert_sdf_samples_to_ply`` writes it
    (vertex x, y, z float; face ``list uchar int vertex_indices``)."""
    verts = np.asarray(verts, "<f4")
    faces = np.asarray(faces, "<i4")
    head = ("ply\nformat binary_little_endian 1.0\n"
            f"element vertex {len(verts)}\nproperty float x\nproperty float y\nproperty float z\n"
            f"element face {len(faces)}\nproperty list uchar int vertex_indices\nend_header\n")
    rec = np.zeros(len(faces), dtype=[("n", "u1"), ("v", "<i4", (3,))])
    rec["n"] = 3
    rec["v"] = faces
    with open(path, "wb") as f:
        f.write(head.encode("ascii"))
        f.write(verts.tobytes())
        f.write(rec.tobytes())


def read_ply(path: str):
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode("ascii").split("\n")
    nv = int([l for l in head if l.startswith("element vertex")][0].split()[-1])
    nf = int([l for l in head if l.startswith("element face")][0].split()[-1])
    verts = np.frombuffer(data, "<f4", nv * 3, end).reshape(nv, 3)
    rec = np.frombuffer(data, [("n", "u1"), ("v", "<i4", (3,))], nf, end + nv * 12)
    assert (rec["n"] == 3).all()
    return verts, rec["v"].astype(np.int32)
