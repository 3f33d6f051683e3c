"""Microbenchmark of the training GEMM shapes (config 2, B = 1000 padded to 1024; C19 1M rows):
ldm_gemm_bf16 per tile shape vs the generic ldm_linear MFMA path vs torch.mm (hipBLASLt) on
the same bf16 operands.  HIP events over REPS back-to-back launches, after a warm-up.
Prints one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops, _capi as capi  # noqa: E402

dev = torch.device("cuda", 0)
REPS = int(os.environ.get("REPS", "50"))
SHAPES = [(1024, 1024, 2048), (1024, 2048, 1024), (1024, 1024, 1024), (1024, 256, 1024),
          (256, 1024, 1024), (1024, 1024, 128), (1024, 1024, 4096)]
if os.environ.get("BIG"):
    SHAPES += [(1 << 20, 512, 512), (512, 512, 1 << 20)]
if os.environ.get("SHAPE"):          # e.g. SHAPE=1024,1024,2048 (profiling one shape)
    SHAPES = [tuple(int(v) for v in os.environ["SHAPE"].split(","))]
TILES = tuple(int(v) for v in os.environ.get("TILES", "1,3,4,5,6,8,9").split(","))
NO_REF = bool(os.environ.get("NO_REF"))
OUT = os.environ.get("OUT", "c")     # epilogue outputs: none | c | cb | cbt | all


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS * 1e3   # us


g = torch.Generator(device=dev).manual_seed(0)
for (M, N, K) in SHAPES:
    PAD = int(os.environ.get("PAD", "0"))         # extra row pitch (elements): L2 channel spread
    A = torch.randn(M, K + PAD, device=dev, generator=g).bfloat16()[:, :K]
    B = torch.randn(N, K + PAD, device=dev, generator=g).bfloat16()[:, :K]
    C = torch.empty(M, N, device=dev)
    fl = 2.0 * M * N * K
    res = {"M": M, "N": N, "K": K, "splitk": int(os.environ.get("SPLITK", "1")), "pad": PAD}
    reps = REPS if M * N * K < 1 << 34 else 5
    Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    CbT = torch.empty(N, M, device=dev, dtype=torch.bfloat16)
    cs = torch.empty((M + 31) // 32, N, device=dev)
    # adfwd / adbwd: the auto-decoder's big products (C19): ReLU with the bf16
    # output in both layouts (the transposed one k-blocked by 8192), and the ReLU backward with
    # the mask operand, both layouts and the 32-row column sums
    CbTb = torch.empty((M + 8191) // 8192 * N * 8192, device=dev, dtype=torch.bfloat16)
    Rb = torch.randn(M, N, device=dev, generator=g).bfloat16() if OUT == "adbwd" else None
    outs = {"none": dict(colsum=cs), "c": dict(C=C), "cb": dict(Cb=Cb), "cbt": dict(CbT=CbT),
            "all": dict(C=C, Cb=Cb, CbT=CbT, colsum=cs),
            "adfwd": dict(mode="relu", Cb=Cb, CbT=CbTb, ct_blk=8192),
            "adbwd": dict(mode="relu_bwd", Rb=Rb, Cb=Cb, CbT=CbTb, ct_blk=8192, colsum=cs)}[OUT]
    res["out"] = OUT
    SPLIT = int(os.environ.get("SPLITK", "1"))      # emulate split-K: one problem per K slice
    parts = [torch.empty(M, N, device=dev) for _ in range(SPLIT)] if SPLIT > 1 else None
    for tile in TILES:
        if SPLIT > 1:
            ks = K // SPLIT
            probs = [ops.gemm_problem([(A[:, i * ks:(i + 1) * ks], B[:, i * ks:(i + 1) * ks])],
                                      M, N, C=parts[i]) for i in range(SPLIT)]
            args = ops.gemm_args(probs, tile)
        else:
            args = ops.gemm_args([ops.gemm_problem([(A, B)], M, N, **outs)], tile)
        us = timed(lambda: ops.gemm_launch(args, dev))
        res[f"gemm_t{tile}_us"] = round(us, 2)
        res[f"gemm_t{tile}_tflops"] = round(fl / us / 1e6, 1)
        if os.environ.get("CHECK") and SPLIT == 1 and "C" in outs:   # this tile's fp32 result
            ref = A.float() @ B.float().T
            res[f"gemm_t{tile}_err"] = float((C - ref).abs().max())
            del ref
    if NO_REF:
        print(json.dumps(res), flush=True)
        continue
    ref = A.float() @ B.float().T
    ops.gemm([ops.gemm_problem([(A, B)], M, N, C=C)])
    res["max_err"] = float((C - ref).abs().max())
    us = timed(lambda: torch.mm(A, B.T))
    res["torch_mm_us"], res["torch_mm_tflops"] = round(us, 2), round(fl / us / 1e6, 1)
    if os.environ.get("GRAPH_REF"):      # hipBLASLt device time: torch.mm replayed from a graph
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        n_in = 20 if reps > 5 else 2
        torch.mm(A, B.T, out=Cm)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(n_in):
                torch.mm(A, B.T, out=Cm)
        us = timed(lambda: gr.replay()) / n_in
        res["torch_mm_graph_us"], res["torch_mm_graph_tflops"] = round(us, 2), round(fl / us / 1e6, 1)
    if M * N * K < 1 << 34:
        Af = A.float()
        us = timed(lambda: ops.linear(Af, B, C, compute=capi.COMPUTE_BF16))
        res["ldm_linear_us"], res["ldm_linear_tflops"] = round(us, 2), round(fl / us / 1e6, 1)
    print(json.dumps(res), flush=True)
