"""CPU check of the index algebra of ldm_conv1d's direct staging (csrc/unet.hip fast_x_* /
fast_w_*, make_plan): for every tap geometry the launch kernel takes, the window items cover
every window position exactly once with the right source element (or zero padding), and the
weight items cover every (row, tap, vector) of the LDS image exactly once.  The GPU tests
(tests/test_gpu_unet.py *_direct cases, and the loop == graph bitwise tests, whose loop runs the
generic staging) check the values; this checks the coverage at many more sizes, without a GPU."""
import itertools

import pytest


def ilog2(x):
    lg = 0
    while (1 << lg) < x:
        lg += 1
    return lg


def plan(TP, C, ksize, stride, mode, epv=8):
    cinp = (C + 15) & ~15
    win = (TP - 1) * stride + ksize
    span = win // 2 + 3 if mode == 1 else win + 2
    lgng = ilog2(span // 4 + 1)
    return dict(cinp=cinp, win=win, lgng=lgng, nx=(cinp // 4) << lgng,
                lgv=ilog2(cinp // epv), nw=16 * ksize * (cinp // epv))


def window_writes(TP, C, L_in, ksize, stride, pad, mode, pos0):
    """{(j, column): source (ci, sp) or None (zero)} as fast_x_store writes it."""
    p = plan(TP, C, ksize, stride, mode)
    pstart = pos0 * stride - pad
    s0 = (pstart >> 1) if mode == 1 else pstart
    a0 = s0 & ~3
    out = {}
    for i in range(p["nx"]):
        gi, q = i & ((1 << p["lgng"]) - 1), i >> p["lgng"]
        sp0 = a0 + 4 * gi
        inb = 0 <= sp0 < L_in
        for e in range(4):
            for r in (0, 1) if mode == 1 else (0,):
                j = (2 * (sp0 + e) + r if mode == 1 else sp0 + e) - pstart
                if not 0 <= j < p["win"]:
                    continue
                for m in range(4):
                    ci = 16 * (q >> 2) + (q & 3) + 4 * m
                    col = 4 * q + m
                    key = (j, col)
                    assert key not in out, f"position {j} column {col} written twice"
                    src = (ci, sp0 + e) if inb and ci < C else None
                    out[key] = src
    return p, out


def perm16(ci):
    return (ci & ~15) | ((ci & 3) << 2) | ((ci >> 2) & 3)


GEOMS = [(3, 1, 1, 0), (3, 2, 1, 0), (4, 2, 1, 0), (1, 1, 0, 0), (3, 1, 1, 1)]


@pytest.mark.parametrize("TP", [16, 32, 64])
@pytest.mark.parametrize("geom", GEOMS, ids=["k3s1", "k3s2", "k4s2", "k1", "k3up2"])
def test_window_items_cover_window_exactly_once(TP, geom):
    ksize, stride, pad, mode = geom
    for C, L_in in [(1, 64), (16, 32), (20, 128), (64, 256), (128, 1024)]:
        L_src = 2 * L_in if mode == 1 else L_in
        L_out = (L_src + 2 * pad - ksize) // stride + 1
        for pos0 in sorted({0, TP, (L_out // TP) * TP - TP, (L_out // TP) * TP}):
            if pos0 < 0:
                continue
            p, out = window_writes(TP, C, L_in, ksize, stride, pad, mode, pos0)
            pstart = pos0 * stride - pad
            inv = {perm16(c): c for c in range(p["cinp"])}
            for j in range(p["win"]):
                for col in range(p["cinp"]):
                    assert (j, col) in out, f"C={C} L={L_in} pos0={pos0}: ({j}, {col}) unwritten"
                    pu = pstart + j                          # position in the (upsampled) row
                    ci = inv[col]
                    want = None
                    if ci < C and 0 <= pu < L_src:
                        want = (ci, pu >> 1 if mode == 1 else pu)
                    assert out[(j, col)] == want, (C, L_in, pos0, j, col, out[(j, col)], want)


@pytest.mark.parametrize("epv", [4, 8])
def test_weight_items_cover_image_exactly_once(epv):
    for C, ksize in itertools.product([1, 16, 32, 64, 128, 256], [1, 3, 4]):
        p = plan(16, C, ksize, 1, 0, epv)
        seen = set()
        for i in range(p["nw"]):
            v, co, k = i & ((1 << p["lgv"]) - 1), (i >> p["lgv"]) & 15, i >> (p["lgv"] + 4)
            key = (co, k, v)
            assert key not in seen
            seen.add(key)
        assert seen == {(co, k, v) for co in range(16) for k in range(ksize)
                        for v in range(p["cinp"] // epv)}
