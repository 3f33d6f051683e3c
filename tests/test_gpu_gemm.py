"""ldm_gemm_bf16 (csrc/gemm_bf16.hip) on the MI355X against fp64 torch on the same bf16
operands: every epilogue mode, K segments, several problems per launch, ragged M / N, the
M_valid row mask, bf16 / transposed outputs, column-sum and loss partials, every tile shape.

Tolerances: the fp64 product of the bf16 operands is the reference; fp32 accumulation of K
products of O(1) values errs by ~1e-7 * sqrt(K) * |terms|, so 2e-6 * sqrt(K) * 4 absolute on
fp32 outputs; bf16 outputs are compared after rounding the reference the same way (RNE), with
one bf16 ulp of slack for values that sit on a rounding boundary."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


def _rand(shape, g, dev, scale=1.0):
    return (torch.randn(shape, generator=g) * scale).to(dev)


def _ref(segs):
    return sum(A.double() @ B.double().T for A, B in segs)


def _bf_close(got, want, tol):
    """bf16 output vs an fp64 reference: within the fp32-accumulation tolerance plus one bf16
    rounding step of the value."""
    w = want.double()
    return bool(((got.double() - w).abs() <= tol + w.abs() * 2 ** -8).all())


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 20, 21, 22, 23, 24, 25, 26])
@pytest.mark.parametrize("M,N,Ks", [(1000, 1024, (2048,)), (64, 64, (64,)), (130, 70, (128, 64)),
                                    (1024, 256, (1024,)), (96, 2048, (256, 128, 64, 512))])
def test_gemm_store_segments_tiles(dev, tile, M, N, Ks):
    from ldm_sdf import ops, LdmError
    g = torch.Generator().manual_seed(M * 7 + N + len(Ks) * 13 + tile)
    segs = [(_rand((M, K), g, dev).bfloat16(), _rand((N, K), g, dev).bfloat16()) for K in Ks]
    if tile >= 20 and any(K % 128 for K in Ks):      # 128-deep stages: K must fit them
        with pytest.raises(LdmError):
            ops.gemm([ops.gemm_problem(segs, M, N, C=torch.zeros(M, N, device=dev))], tile=tile)
        return
    bias = _rand((N,), g, dev)
    Mp = (M + 3) // 4 * 4
    C = torch.full((M, N), 7.0, device=dev)
    Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    CbT = torch.zeros(N, Mp, device=dev, dtype=torch.bfloat16)
    Aseg = [(torch.cat([A, torch.zeros(Mp - M, A.shape[1], device=dev, dtype=A.dtype)]), B)
            for A, B in segs]
    cs = torch.zeros((Mp + 31) // 32, N, device=dev)
    ops.gemm([ops.gemm_problem(Aseg, Mp, N, M_valid=M, bias=bias, C=torch.cat(
        [C, torch.zeros(Mp - M, N, device=dev)]) if Mp != M else C, Cb=None, CbT=CbT,
        colsum=cs)], tile=tile)
    # run again with exactly M rows for the row-major outputs
    ops.gemm([ops.gemm_problem(segs, M, N, bias=bias, C=C, Cb=Cb)], tile=tile)
    torch.cuda.synchronize()
    want = _ref(segs) + bias.double()
    tol = 2e-6 * math.sqrt(sum(Ks)) * 4
    assert (C.double() - want).abs().max() < tol
    assert _bf_close(Cb, want, tol)
    assert _bf_close(CbT[:, :M].T, want, tol)
    assert bool((CbT[:, M:] == 0).all())
    csw = torch.zeros_like(cs, dtype=torch.float64)
    for r in range(cs.shape[0]):
        csw[r] = want[r * 32:(r + 1) * 32].sum(0)
    assert (cs.double() - csw).abs().max() < tol * 32


@pytest.mark.parametrize("tile", [0, 16, 21])
@pytest.mark.parametrize("mode", ["silu", "resid_silu", "relu", "accum", "add_r", "dgrad_silu",
                                  "loss", "relu_bwd"])
def test_gemm_epilogues(dev, mode, tile):
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(hash(mode) % 1000)
    M, N, K = 200, 192, 384
    Mv = 190
    A = _rand((M, K), g, dev).bfloat16()
    B = _rand((N, K), g, dev, 0.1).bfloat16()
    bias = _rand((N,), g, dev)
    R = _rand((M, N), g, dev)
    Pin = _rand((M, N), g, dev)
    Rb = _rand((M, N), g, dev).bfloat16()
    Rb[::7] = 0.0                              # +0 and -0 both mask the gradient
    Rb[3::11] = -0.0
    C0 = _rand((M, N), g, dev)
    C = C0.clone()
    P = torch.zeros(M, N, device=dev)
    Cb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    CbT = torch.zeros(N, M, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros((M + 31) // 32, N, device=dev)
    lp = torch.zeros((M + 31) // 32, (N + 31) // 32, device=dev)
    kw = dict(bias=bias, C=C, Cb=Cb, CbT=CbT, colsum=cs, M_valid=Mv)
    if mode in ("silu", "resid_silu"):
        kw["P"] = P
    if mode in ("resid_silu", "add_r", "dgrad_silu"):
        kw["R"] = R
    if mode in ("dgrad_silu", "loss"):
        kw["P_in"] = Pin
    if mode == "loss":
        kw["loss_part"] = lp
        kw["scale"] = 0.37
    if mode == "relu_bwd":
        kw["Rb"] = Rb
    ops.gemm([ops.gemm_problem([(A, B)], M, N, mode=mode, **kw)], tile=tile)
    torch.cuda.synchronize()
    pre = A.double() @ B.double().T + bias.double()
    sig = torch.sigmoid
    Rd, Pd, C0d = R.double(), Pin.double(), C0.double()
    dh = None
    if mode == "silu":
        out = pre * sig(pre)
    elif mode == "resid_silu":
        out = Rd + pre * sig(pre)
    elif mode == "relu":
        out = pre.clamp_min(0)
    elif mode == "accum":
        out = C0d + pre
    elif mode == "add_r":
        out = Rd + pre
    elif mode == "dgrad_silu":
        dh = Rd + pre
        s = sig(Pd)
        out = dh * s * (1 + Pd * (1 - s))
    elif mode == "relu_bwd":
        out = torch.where(Rb.double() > 0, pre, torch.zeros_like(pre))
    else:
        d = pre - Pd
        out = 0.37 * d
    live = torch.arange(M, device=dev)[:, None] < Mv
    out = torch.where(live, out, torch.zeros_like(out))
    tol = 2e-6 * math.sqrt(K) * 4 * 4
    # fp32 outputs: live rows computed, padding rows (>= M_valid) left as they were
    Cw = dh if mode == "dgrad_silu" else out
    assert (C[:Mv].double() - Cw[:Mv]).abs().max() < tol, mode
    assert torch.equal(C[Mv:], C0[Mv:])
    assert _bf_close(Cb, out, tol)
    assert _bf_close(CbT.T, out, tol)
    assert bool((Cb[Mv:] == 0).all()) and bool((CbT[:, Mv:] == 0).all())
    if mode in ("silu", "resid_silu"):
        assert (P[:Mv].double() - pre[:Mv]).abs().max() < tol
        assert bool((P[Mv:] == 0).all())
    csw = torch.stack([out[r * 32:(r + 1) * 32].sum(0) for r in range(cs.shape[0])])
    assert (cs.double() - csw).abs().max() < tol * 32
    if mode == "loss":
        d2 = torch.where(live, (pre - Pd) ** 2, torch.zeros_like(pre))
        lw = torch.stack([torch.stack([d2[r * 32:(r + 1) * 32, c * 32:(c + 1) * 32].sum()
                                       for c in range(lp.shape[1])]) for r in range(lp.shape[0])])
        assert (lp.double() - lw).abs().max() < 1e-4 * lw.abs().max()


def test_gemm_grouped_problems(dev):
    """Four problems of different shapes and modes in one launch == four launches."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(77)
    shapes = [(1024, 1024, 1024), (256, 1024, 1024), (1024, 128, 1024), (64, 2048, 192)]
    probs, outs, refs, keep = [], [], [], []
    for (M, N, K) in shapes:
        A = _rand((M, K), g, dev).bfloat16()
        B = _rand((N, K), g, dev).bfloat16()
        C = torch.zeros(M, N, device=dev)
        keep += [A, B]                  # the problem holds raw pointers: keep the operands alive
        probs.append(ops.gemm_problem([(A, B)], M, N, C=C))
        outs.append(C)
        refs.append(A.double() @ B.double().T)
    ops.gemm(probs)
    torch.cuda.synchronize()
    for (M, N, K), C, w in zip(shapes, outs, refs):
        assert (C.double() - w).abs().max() < 2e-6 * math.sqrt(K) * 4, (M, N, K)


def test_gemm_rejects_bad_args(dev):
    from ldm_sdf import ops, LdmError
    A = torch.zeros(64, 100, device=dev, dtype=torch.bfloat16)
    B = torch.zeros(64, 100, device=dev, dtype=torch.bfloat16)
    with pytest.raises(LdmError):                     # K not a multiple of 64
        ops.gemm([ops.gemm_problem([(A, B)], 64, 64, C=torch.zeros(64, 64, device=dev))])
    A = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    with pytest.raises(LdmError):                     # resid_silu without R
        ops.gemm([ops.gemm_problem([(A, A)], 64, 64, mode="resid_silu",
                                   C=torch.zeros(64, 64, device=dev))])


@pytest.mark.parametrize("tile", [0, 4, 16, 20, 26])
@pytest.mark.parametrize("ks,mode", [(2, "store"), (8, "store"), (4, "accum")])
def test_gemm_split_k(dev, tile, ks, mode):
    """Split-K (C19's weight gradients G^T X over ~1M samples): slices write raw partials to
    ws, a second kernel sums them in slice order and applies bias / ACCUM.  Ragged M / N and an
    M_valid row mask; the result is deterministic (two launches give the same bits)."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(ks * 31 + tile)
    M, N, K, Mv = 330, 200, 128 * ks * 3, 321
    A = _rand((M, K), g, dev).bfloat16()
    B = _rand((N, K), g, dev).bfloat16()
    bias = _rand((N,), g, dev)
    C0 = _rand((M, N), g, dev)
    ws = torch.full((ks * M * N,), float("nan"), device=dev)
    outs = []
    for _ in range(2):
        C = C0.clone()
        ops.gemm([ops.gemm_problem([(A, B)], M, N, mode=mode, M_valid=Mv, bias=bias, C=C,
                                   k_split=ks, ws=ws)], tile=tile)
        outs.append(C)
    torch.cuda.synchronize()
    want = A.double() @ B.double().T + bias.double()
    if mode == "accum":
        want = want + C0.double()
    C = outs[0]
    assert (C[:Mv].double() - want[:Mv]).abs().max() < 2e-6 * math.sqrt(K) * 4 * 2
    assert torch.equal(C[Mv:], C0[Mv:])                  # padding rows untouched
    assert torch.equal(outs[0], outs[1])


def test_gemm_persistent_many_tiles(dev):
    """Persistent tiles (16 / 17 / 18) when the launch has several tiles per resident workgroup:
    K segments of different lengths, two problems with different k-step counts, a ragged M, the
    RELU_BWD mask and both bf16 layouts -- equal to the one-tile-per-workgroup kernel bit for
    bit (same k order, same epilogue)."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(5)
    M1, N1, M2, N2 = 40000, 384, 9000, 256
    A1 = _rand((M1, 128), g, dev).bfloat16()
    A1b = _rand((M1, 64), g, dev).bfloat16()
    B1 = _rand((N1, 128), g, dev, 0.1).bfloat16()
    B1b = _rand((N1, 64), g, dev, 0.1).bfloat16()
    A2 = _rand((M2, 512), g, dev).bfloat16()
    B2 = _rand((N2, 512), g, dev, 0.1).bfloat16()
    Rb = _rand((M2, N2), g, dev).bfloat16()
    bias = _rand((N1,), g, dev)
    res = {}
    for tile in (4, 16, 17, 18):
        C1 = torch.zeros(M1, N1, device=dev)
        Cb1 = torch.zeros(M1, N1, device=dev, dtype=torch.bfloat16)
        C2 = torch.zeros(M2, N2, device=dev)
        CbT2 = torch.zeros(N2, M2, device=dev, dtype=torch.bfloat16)
        ops.gemm([ops.gemm_problem([(A1, B1), (A1b, B1b)], M1, N1, mode="relu", bias=bias,
                                   C=C1, Cb=Cb1),
                  ops.gemm_problem([(A2, B2)], M2, N2, mode="relu_bwd", Rb=Rb, C=C2, CbT=CbT2,
                                   M_valid=M2 - 37)], tile=tile)
        torch.cuda.synchronize()
        res[tile] = (C1, Cb1, C2, CbT2)
    want1 = (A1.double() @ B1.double().T + A1b.double() @ B1b.double().T + bias.double()).clamp_min(0)
    assert (res[16][0].double() - want1).abs().max() < 2e-6 * math.sqrt(192) * 4
    for tile in (16, 17, 18):
        for got, ref in zip(res[tile], res[4]):
            assert torch.equal(got, ref), tile


def test_gemm_blocked_transpose_and_sliced_split_k(dev):
    """C19's sample-axis operands: a forward writes CbT k-blocked ([M/KT][N][KT], ct_blk),
    and a weight-gradient product sums over the blocks as split-K slices (slices = block
    strides).  Equal to the plain transposed layout / the fp64 product of the same bf16 values."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(11)
    M, N, K, KT, Mv = 2048, 96, 128, 256, 2000
    A = _rand((M, K), g, dev).bfloat16()
    B = _rand((N, K), g, dev).bfloat16()
    plain = torch.zeros(N, M, device=dev, dtype=torch.bfloat16)
    blocked = torch.full((M // KT, N, KT), 3.0, device=dev, dtype=torch.bfloat16)
    ops.gemm([ops.gemm_problem([(A, B)], M, N, mode="relu", M_valid=Mv, CbT=plain)])
    ops.gemm([ops.gemm_problem([(A, B)], M, N, mode="relu", M_valid=Mv, CbT=blocked,
                               ct_blk=KT)])
    torch.cuda.synchronize()
    assert torch.equal(blocked.permute(1, 0, 2).reshape(N, M), plain)
    # weight gradient: G^T [N2][M] (blocked) x X^T [N][M] (blocked) over the M samples
    N2 = 72
    G = _rand((N2, M), g, dev).bfloat16()
    Gb = G.view(N2, M // KT, KT).permute(1, 0, 2).contiguous()
    out = torch.zeros(N2, N, device=dev)
    ks = M // KT
    ws = torch.empty(ks * N2 * N, device=dev)
    ops.gemm([ops.gemm_problem([(Gb[0], blocked[0])], N2, N, C=out, k_split=ks, ws=ws,
                               slices=(N2 * KT, N * KT))])
    torch.cuda.synchronize()
    want = G.double() @ plain.double().T
    assert (out.double() - want).abs().max() < 2e-6 * math.sqrt(M) * 4 * 4


@pytest.mark.parametrize("tile", [0, 4, 15, 20, 24])
@pytest.mark.parametrize("mode", ["store", "silu", "resid_silu", "relu", "accum", "add_r",
                                  "dgrad_silu", "loss", "relu_bwd"])
def test_gemm_lds_epilogue_bitwise_vs_accumulator_layout(dev, mode, tile):
    """The LDS-transposed epilogue (16-byte row-major stores) against the accumulator-layout
    stores it replaced, on the same problem: row strides of N + 1 elements (not a multiple of
    4) force every block onto the old path.  Every output must match bit for bit."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(hash(mode) % 997 + tile)
    M, N, K = 200, 192, 384
    Mv = 190
    A = _rand((M, K), g, dev).bfloat16()
    B = _rand((N, K), g, dev, 0.1).bfloat16()
    bias = _rand((N,), g, dev)
    R = _rand((M, N), g, dev)
    Pin = _rand((M, N), g, dev)
    Rb = _rand((M, N), g, dev).bfloat16()
    Rb[::7] = 0.0
    C0 = _rand((M, N), g, dev)

    def run(pad):
        def f32(src=None):
            t = torch.zeros(M, N + pad, device=dev)
            if src is not None:
                t[:, :N] = src
            return t[:, :N]
        C = f32(C0)
        P = f32()
        Cb = torch.zeros(M, N + pad, device=dev, dtype=torch.bfloat16)[:, :N]
        CbT = torch.zeros(N, M, device=dev, dtype=torch.bfloat16)
        cs = torch.zeros((M + 31) // 32, N, device=dev)
        lp = torch.zeros((M + 31) // 32, (N + 31) // 32, device=dev)
        kw = dict(bias=bias, C=C, Cb=Cb, CbT=CbT, colsum=cs, M_valid=Mv)
        if mode in ("silu", "resid_silu"):
            kw["P"] = P
        if mode in ("resid_silu", "add_r", "dgrad_silu"):
            kw["R"] = f32(R)
        if mode in ("dgrad_silu", "loss"):
            kw["P_in"] = f32(Pin)
        if mode == "loss":
            kw["loss_part"] = lp
            kw["scale"] = 0.37
        if mode == "relu_bwd":
            Rbp = torch.zeros(M, N + pad, device=dev, dtype=torch.bfloat16)
            Rbp[:, :N] = Rb
            kw["Rb"] = Rbp[:, :N]
        ops.gemm([ops.gemm_problem([(A, B)], M, N, mode=mode, **kw)], tile=tile)
        torch.cuda.synchronize()
        return [x.contiguous() for x in (C, P, Cb, CbT, cs, lp)]

    new, old = run(0), run(1)
    for a, b, name in zip(new, old, ("C", "P", "Cb", "CbT", "colsum", "loss_part")):
        assert torch.equal(a, b), (mode, tile, name)
