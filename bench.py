"""Benchmark: SDF queries/s on 256^3 grids (+ DDPM sample steps/s), 1..8 MI355X.

One "step" = decode of ``--batch`` synthetic shapes on a ``--grid``^3 grid (config 4:
B=64, 256^3), z-slab sharded over the ranks with per-shape RCCL all-gathers of the volume
(SURVEY.md §8(e)).  Total work is fixed as N grows (``scaling: strong``); ``value`` =
all queries of the step / max-over-ranks step time.

Launch: ``python bench.py`` (1 GPU), ``torchrun --nproc-per-node N bench.py --gpus N``, or
``python bench.py --gpus N`` (spawns the N ranks itself through torch.distributed.run, as a
child process started before anything touches the GPU).  Rank 0 prints ONE JSON line.
Extra objects: ``roofline`` (dominant kernel, HIP events on its stream), ``cpu_baseline``
(oracle/ref_cpu.py fp32 on this host's cores, bounded sample), ``ddpm`` (1000-step sampling
of 8 latents, steps/s, + config 3 end to end), ``config5``, ``train`` (config 2), ``mc``,
``autodecoder``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FLOPS_PER_QUERY = 2 * (3 * 512 + 2 * 512 * 512 + 512 * 253 + 256 * 512 + 3 * 512 * 512 + 512)
PEAK_TFLOPS = {"bf16": 2516.6, "fp16": 2516.6, "fp32": 157.3}   # MI355X dense (MICROARCH guide)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ddpm", action="store_true")
    ap.add_argument("--ddpm-batch", type=int, default=8)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--train-steps", type=int, default=100)
    ap.add_argument("--no-config5", action="store_true",
                    help="skip config 5 (1D-UNet sampling on 1024-d latents -> fp16 decode "
                         "of a 512^3 grid with the widen-skip decoder)")
    ap.add_argument("--c5-batch", type=int, default=1)
    ap.add_argument("--no-mc", action="store_true",
                    help="skip C18 (marching cubes of one decoded 256^3 volume)")
    ap.add_argument("--no-autodecoder", action="store_true",
                    help="skip C19 (DeepSDF auto-decoder training at 64 shapes x 16384 samples)")
    ap.add_argument("--ad-steps", type=int, default=5)
    ap.add_argument("--no-config3", action="store_true",
                    help="skip config 3 (sample(8) -> decode 128^3, timed end to end; its "
                         "decode is a dec_fs_kernel launch of another size in a profile)")
    ap.add_argument("--shapes-per-group", type=int, default=0,
                    help="multi-GPU decode: shapes per gather group (0: ceil(B/8))")
    return ap.parse_args()


def host_cores() -> int:
    """Cores this job may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU box
    exposes the whole machine in the mask but allots each 1-GPU job a 16-core share)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_fields(cores: int) -> dict:
    """CPU model, threads used and cores available, for every ``cpu_baseline``."""
    return {"cores": cores, "threads": torch.get_num_threads(), "cpu_model": cpu_model(),
            "affinity_cpus": len(os.sched_getaffinity(0))}


def cpu_baseline_decode(grid: int, budget_s: float):
    """oracle decode (torch CPU fp32, this job's cores) of whole z-slices of the grid until
    ``budget_s`` of work; q/s is flat in N."""
    from oracle import ref_cpu as R
    cores = host_cores()
    torch.set_num_threads(cores)
    p = R.make_decoder_params(seed=1234, dtype=torch.float32)
    z = torch.randn(1, 256, generator=torch.Generator().manual_seed(0)) * 0.1
    pts = 0
    t0 = time.perf_counter()
    k = 0
    while k < grid:
        R.decode_grid(p, z, grid, k, k + 1)
        pts += grid * grid
        k += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": pts / dt, "unit": "queries/s", "kind": "port", **cpu_fields(cores),
            "sample": f"{k} z-slices x {grid}x{grid} of the {grid}^3 grid ({pts} queries), "
                      f"1 shape, fp32 torch-CPU oracle, {dt:.1f}s"}


def cpu_baseline_sampling(budget_s: float, B: int):
    from oracle import ref_cpu as R
    torch.set_num_threads(host_cores())
    p = R.make_denoiser_params(seed=4321, dtype=torch.float32)
    tab = R.ddpm_tables()
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128))
    x = torch.randn(B, 256)
    noise = torch.randn(1000, B, 256)
    t0 = time.perf_counter()
    steps = 0
    with torch.inference_mode():
        for t in range(999, -1, -1):
            eps = R.denoiser_forward(p, x, torch.full((B,), t), emb)
            x = R.ddpm_step(tab, x, eps, noise[t], t)
            steps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "steps/s", "kind": "port",
            **cpu_fields(host_cores()),
            "sample": f"{steps} reverse steps, B={B}, fp32 torch-CPU oracle, {dt:.1f}s"}


def cpu_baseline_train(budget_s: float, batch: int = 1000):
    """Config 2 on the CPU: the fp32 oracle training step (q_sample -> denoiser -> eps-MSE ->
    autograd backward, oracle/ref_cpu.py train_step's math) + torch AdamW on the fp32
    parameters, batch ``batch`` on 1000 latents, this job's cores; steps until ``budget_s``."""
    from oracle import ref_cpu as R
    torch.set_num_threads(host_cores())
    p = R.make_denoiser_params(seed=4321, dtype=torch.float32)
    params = p.map(lambda w: w.detach().clone().requires_grad_(True))
    leaves = [params.Wt1, params.bt1, params.Wt2, params.bt2, params.Win, params.bin,
              params.Wout, params.bout] + list(params.Wblk) + list(params.bblk)
    opt = torch.optim.AdamW(leaves, lr=1e-4, weight_decay=0.0)
    tab = R.ddpm_tables()
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128))
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(1000, 256, generator=g) * 0.5
    steps, t0 = 0, time.perf_counter()
    while True:
        t = torch.randint(0, 1000, (batch,), generator=g)
        eps = torch.randn(batch, 256, generator=g)
        x0 = lat[:batch]
        with torch.enable_grad():
            xt = R.q_sample(tab, x0, eps, t)
            loss = R.eps_mse_loss(R.denoiser_forward(params, xt, t, emb), eps)
            opt.zero_grad(set_to_none=True)
            loss.backward()
        opt.step()
        steps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "steps/s", "kind": "port",
            **cpu_fields(host_cores()),
            "sample": f"{steps} fp32 torch-CPU oracle training steps (autograd + AdamW), "
                      f"batch {batch}, {dt:.1f}s"}


def cpu_baseline_unet(budget_s: float, B: int):
    """Config 5's sampler on the CPU: the fp32 oracle UNet (oracle/ref_unet.py) reverse steps."""
    from oracle import ref_cpu as R
    from oracle import ref_unet as U
    torch.set_num_threads(host_cores())
    up = U.make_unet_params(seed=2468, dtype=torch.float32)
    tab = R.ddpm_tables()
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128))
    x = torch.randn(B, 1024)
    noise = torch.randn(1000, B, 1024)
    t0 = time.perf_counter()
    steps = 0
    with torch.inference_mode():
        for t in range(999, -1, -1):
            eps = U.unet_forward(up, x, torch.full((B,), t), emb)
            x = R.ddpm_step(tab, x, eps, noise[t], t)
            steps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "steps/s", "kind": "port",
            **cpu_fields(host_cores()),
            "sample": f"{steps} reverse steps of the 1D-UNet (D=1024), B={B}, fp32 torch-CPU "
                      f"oracle, {dt:.1f}s"}


def bench_mc(vol, args):
    """C18: marching cubes of one decoded volume (shape 0 of the step), on the GPU, with the
    oracle (numpy) timed on the same volume as the CPU baseline."""
    import ldm_sdf
    from ldm_sdf import _capi as capi
    N = vol.shape[-1]
    ws = torch.empty(capi.load().ldm_mc_workspace_bytes(N), device=vol.device, dtype=torch.uint8)
    v, f = ldm_sdf.marching_cubes(vol, ws=ws)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        v, f = ldm_sdf.marching_cubes(vol, ws=ws)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    nbytes = N ** 3 * 4 + v.shape[0] * 12 + f.shape[0] * 12
    res = {"metric": "marching cubes of one decoded volume", "grid": N,
           "vertices": int(v.shape[0]), "faces": int(f.shape[0]), "ms_per_mesh": dt * 1e3,
           "note": "wall time incl. the one count read-back between the passes",
           "roofline": {"bound": "hbm", "achieved": nbytes / dt / 1e9, "peak": 8000.0,
                        "unit": "GB/s", "frac": nbytes / dt / 8e12,
                        "algorithmic_bytes": nbytes}}
    if not args.no_cpu:
        from oracle import ref_mc as M
        vn = vol.cpu().numpy()
        t1 = time.perf_counter()
        M.marching_cubes(vn)
        res["cpu_baseline"] = {"value": 1.0 / (time.perf_counter() - t1), "unit": "meshes/s",
                               "kind": "port", **cpu_fields(1), "cores": 1,
                               "sample": f"oracle/ref_mc.py (numpy) on the same {N}^3 volume"}
    res["value"] = 1.0 / dt
    res["unit"] = "meshes/s"
    return res


FLOPS_PER_QUERY_WIDEN = 2 * (3 * 512 + 2 * 512 * 512 + 512 * 512 + 515 * 512 + 3 * 512 * 512
                             + 512)


def bench_autodecoder(args, dev):
    """C19: DeepSDF auto-decoder training steps at the DeepSDF batch (64 scenes x 16384 SDF
    samples = 1,048,576 samples/step), bf16 matrix-core GEMMs, synthetic near-surface sphere
    samples.  CPU baseline: the fp32 oracle step (torch autograd) on a 1 x 4096 sample."""
    import ldm_sdf
    S, P = 64, 16384
    g = torch.Generator(device=dev).manual_seed(7)
    radii = 0.3 + 0.5 * torch.rand(S, device=dev, generator=g)
    d = torch.randn(S, P, 3, device=dev, generator=g)
    d = d / d.norm(dim=2, keepdim=True)
    r = radii[:, None] + 0.05 * torch.randn(S, P, device=dev, generator=g)
    xyz = d * r[..., None]
    sdf = xyz.norm(dim=2) - radii[:, None]
    dec = ldm_sdf.SDFDecoder(seed=1234)
    dec.weights[8] = dec.weights[8] * 0.01
    # (group=LOCAL: rank 0 only at world > 1, as for config 2)
    from ldm_sdf.dist import LOCAL
    st = ldm_sdf.train_autodecoder(dec, xyz, sdf, steps=1, shapes_per_batch=S,
                                   samples_per_shape=P, dtype="bf16", generator=g, group=LOCAL)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = ldm_sdf.train_autodecoder(dec, xyz, sdf, steps=args.ad_steps, shapes_per_batch=S,
                                   samples_per_shape=P, dtype="bf16", generator=g, state=st,
                                   group=LOCAL)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.ad_steps
    fwd = sum(2 * i * o for (i, o) in ldm_sdf.decoder_layer_dims(256, 512))   # per sample
    res = {"metric": "DeepSDF auto-decoder training steps/sec (64 x 16384 samples)",
           "value": 1.0 / dt, "unit": "steps/s", "ms_per_step": dt * 1e3,
           "samples_per_s": S * P / dt, "flops_per_sample_fwd": fwd,
           "tflops_fwd_bwd": 3 * fwd * S * P / dt / 1e12, "dtype": "bf16",
           "roofline": {"bound": "mfma", "achieved": 3 * fwd * S * P / dt / 1e12,
                        "peak": PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                        "frac": 3 * fwd * S * P / dt / 1e12 / PEAK_TFLOPS["bf16"],
                        "flops_per_step": 3 * fwd * S * P,
                        "note": "3 x forward FLOPs (forward, dX and dW products) of the "
                                "1,048,576 samples over the wall time of a step (every launch "
                                "incl. the loss, latent gradients and Adam)"},
           "loss_first_last": [st.losses[0], st.losses[-1]]}
    if not args.no_cpu:
        from oracle import ref_cpu as R
        from oracle import ref_autodecoder as A
        torch.set_num_threads(host_cores())
        p = R.make_decoder_params(seed=1234, dtype=torch.float32)
        zc = torch.randn(1, 256) / 16
        xc, sc = xyz[:1, :4096].cpu(), sdf[:1, :4096].cpu()
        A.autodecoder_grads(p, zc, xc, sc)
        n, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < min(5.0, args.cpu_seconds):
            A.autodecoder_grads(p, zc, xc, sc)
            n += 1
        sps = n * 4096 / (time.perf_counter() - t1)
        res["cpu_baseline"] = {"value": sps, "unit": "samples/s", "kind": "port",
                               **cpu_fields(host_cores()),
                               "sample": f"{n} fp32 oracle steps (torch autograd) of 1 shape x "
                                         "4096 samples"}
    return res


class SlabTimer:
    """The decode slab function handed to ``dist.decode_sharded`` (or called directly at one
    rank): launches ``ldm_decoder_grid_fwd`` for shapes [b0, b1) of the z-slab [k0, k1) and,
    when ``timed``, brackets the launch with HIP events on the kernel's stream."""

    def __init__(self, desc, beta_fn, N, stream):
        self.desc, self.beta_fn, self.N, self.stream = desc, beta_fn, N, stream
        self.timed = False
        self.events = []          # (start, end, queries of the launch)
        self.beta = None

    def __call__(self, k0, k1, dst, b0, b1):
        from ldm_sdf import ops
        if b0 == 0 or self.beta is None:
            self.beta = self.beta_fn()     # A2 fold once per step (first group)
        if self.timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
        ops.decoder_grid_fwd(self.desc, self.beta[b0:b1], self.N, k0, k1, out=dst)
        if self.timed:
            e1.record(self.stream)
            self.events.append((e0, e1, (b1 - b0) * (k1 - k0) * self.N * self.N))

    def kernel_stats(self):
        """(average launch ms, average queries per launch) over the timed launches."""
        if not self.events:
            return float("nan"), 0
        ms = [a.elapsed_time(b) for a, b, _ in self.events]
        return sum(ms) / len(ms), sum(q for _, _, q in self.events) / len(self.events)


def run_decode_steps(slab, B: int, N: int, *, steps: int, warmup: int, world: int, group,
                     device: torch.device, out: torch.Tensor, sync=None,
                     shapes_per_group=None, on_timed=None, local=None,
                     step_events=None) -> float:
    """The bench's per-rank step loop (shared with the gloo test, tests/test_bench_gloo.py):
    ``warmup`` untimed steps, then barrier + sync, ``steps`` timed steps, sync + barrier, and
    the MAX of the per-rank elapsed times (all-reduce; ``local``, a list, receives this rank's
    own).  One step = the (sharded) decode of B
    shapes on an N^3 grid into ``out``; ``slab(k0, k1, dst, b0, b1)`` computes a slab.
    ``step_events`` (a list, GPU only): receives one (start, end) HIP event pair per timed step,
    recorded on the current stream around it (per-step hipEvent times, median)."""
    from ldm_sdf.dist import decode_sharded
    sync = sync or (lambda: None)

    def step():
        if world == 1:
            slab(0, N, out, 0, B)
        else:
            decode_sharded(slab, B, N, device, group=group, out=out,
                           shapes_per_group=shapes_per_group)

    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier(group)
    sync()
    if on_timed:
        on_timed()
    ev = step_events is not None and device.type == "cuda"
    t0 = time.perf_counter()
    for _ in range(steps):
        if ev:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        step()
        if ev:
            e1.record()
            step_events.append((e0, e1))
    sync()
    if world > 1:
        dist.barrier(group)
    elapsed = time.perf_counter() - t0
    if local is not None:
        local.append(elapsed)           # this rank's own time (before the max over ranks)
    if world > 1:
        tt = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(tt)
    return elapsed


def event_summary(pairs) -> dict:
    """Per-step HIP event times (ms) of the timed steps: median, min, max, mean, count."""
    ms = sorted(a.elapsed_time(b) for a, b in pairs)
    if not ms:
        return None
    return {"median_ms": ms[len(ms) // 2] if len(ms) % 2 else 0.5 * (ms[len(ms) // 2 - 1] +
                                                                        ms[len(ms) // 2]),
            "min_ms": ms[0], "max_ms": ms[-1], "mean_ms": sum(ms) / len(ms), "n": len(ms),
            "source": "hipEvent pair per timed step on the decode stream"}


def rank_breakdown(step_ms: float, kernel_ms: float, group, device) -> dict:
    """Every rank's step time, its slab kernels' time per step (HIP events) and the difference
    -- the part of the all-gathers the kernels did not hide -- gathered from all ranks, with the
    world size and backend the process group reports (tests/test_bench_gloo.py)."""
    loc = torch.tensor([step_ms, kernel_ms], device=device, dtype=torch.float64)
    n = dist.get_world_size(group)
    allv = [torch.zeros_like(loc) for _ in range(n)]
    dist.all_gather(allv, loc, group=group)
    return {"world_seen": n, "backend": dist.get_backend(group),
            "per_rank": [{"rank": r, "step_ms": float(v[0]), "kernel_ms": float(v[1]),
                          "gather_exposed_ms": float(v[0] - v[1])} for r, v in enumerate(allv)]}


def decoder_traffic(queries_per_launch: float):
    """HBM bytes per launch for ``roofline.traffic``: the PMC bytes per query measured at
    B = 64 x 256^3 (profiles/decoder_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE, the MI355X
    guide's gfx950 correction) scaled to this run's queries per launch -- the traffic is
    linear in the queries (4 B written each; the ~62 MB of weight/aux reads per launch are
    <1.5 %).  None when the file is absent."""
    tf = os.path.join(ROOT, "profiles", "decoder_traffic.json")
    if not os.path.exists(tf):
        return None, None
    try:
        j = json.load(open(tf))
        per_q = j["hbm_bytes_per_launch"] / j["queries_per_launch"]
    except (OSError, ValueError, KeyError, ZeroDivisionError):
        return None, None
    return per_q * queries_per_launch, j.get("source", tf)


def handoff_latency():
    """The same-XCD one-way latency of the sampler's 8-byte tagged hand-off, measured by
    scripts/microbench/handoff_latency.hip on an MI355X (median of its reps), from the newest
    profiles/*/handoff_latency.json; None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "handoff_latency.json")))
    if not files:
        return None
    try:
        rows = [json.loads(l) for l in open(files[-1]) if l.strip().startswith("{")]
        same = sorted(r["one_way_ns"] for r in rows if r.get("pair") == "same-XCD" and r["ok"])
    except (OSError, ValueError, KeyError):
        return None
    if not same:
        return None
    return {"one_way_ns": same[len(same) // 2], "source": os.path.relpath(files[-1], ROOT)}


def allgather_latency():
    """Per-layer latency of the sampler's hand-off pattern without its arithmetic: an
    all-gather of 1024 tagged 8-byte granules among one XCD's 32 workgroups, all 8 XCDs at once
    (scripts/microbench/allgather_latency.hip, median of its reps), from the newest
    profiles/*/allgather_latency.json; None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "allgather_latency.json")))
    if not files:
        return None
    try:
        rows = [json.loads(l) for l in open(files[-1]) if l.strip().startswith("{")]
        ph = sorted(r["phase_ns_median"] for r in rows if r["ok"])
    except (OSError, ValueError, KeyError):
        return None
    if not ph:
        return None
    return {"phase_ns": ph[len(ph) // 2], "source": os.path.relpath(files[-1], ROOT)}


def config5(args, rank, world, dev, group, gen):
    """Config 5: 1000-step DDPM sampling of ``--c5-batch`` 1024-d latents with the 1D-UNet
    (bf16 weights, hipGraph) -> fp16 MFMA decode (widen-skip decoder, L=1024) of a 512^3
    grid, z-slab sharded over the ranks + all-gathers.  Decode time = max over ranks."""
    import ldm_sdf
    nb, N = args.c5_batch, 512
    unet = ldm_sdf.UNet1DDenoiser(D=1024, seed=2468)
    sch = ldm_sdf.DDPMSchedule()
    lo, hi = ldm_sdf.dist.batch_shard(nb, rank, world)
    nl = max(1, hi - lo)
    xT = torch.randn(nl, 1024, device=dev, generator=gen)
    noise = torch.randn(1000, nl, 1024, device=dev, generator=gen)

    # the Sampler path: the hipGraph of 1000 steps x 18 ldm_conv1d launches (the
    # round-3 one-launch loop was retired in round 4)
    smp = ldm_sdf.Sampler(unet, sch, nl, dtype="bf16", device=dev)
    smp.run(xT, noise)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        lat = smp.run(xT, noise).clone()
    torch.cuda.synchronize()
    sps = 1000 * reps / (time.perf_counter() - t0)
    latents = ldm_sdf.dist.all_gather_rows(lat[:hi - lo].clone(), nb, group=group) \
        if world > 1 else lat[:nb].clone()
    dec = ldm_sdf.SDFDecoder(1024, seed=1235)            # widen-skip (L + 3 >= H)
    from ldm_sdf import ops
    desc = dec.device_pack("fp16", dev)["desc"]
    out = torch.empty(nb, N, N, N, device=dev)
    stream = torch.cuda.current_stream(dev)
    slab = SlabTimer(desc, lambda: ops.decoder_fold(desc, latents.float().contiguous()), N,
                     stream)
    el = run_decode_steps(slab, nb, N, steps=1, warmup=1, world=world, group=group,
                          device=dev, out=out, sync=torch.cuda.synchronize,
                          on_timed=lambda: setattr(slab, "timed", True))
    kms, qpl = slab.kernel_stats()
    ach = FLOPS_PER_QUERY_WIDEN * qpl / (kms * 1e-3) / 1e12
    wbytes = 2 * sum(v.numel() for k, v in unet.params.items()
                     if not (k.startswith("b") or k.endswith((".b", ".b1", ".b2", ".bs"))
                             or k.startswith("Wt") or k.endswith(".p")))
    res = {"workload": f"config5: {nb} x 1000-step 1D-UNet sampling (D=1024, C=(32,64,128), "
                       f"bf16) -> fp16 decode of a {N}^3 grid (widen-skip, L=1024), "
                       f"z-slab over {world} rank(s)",
           "decode_queries_per_s": nb * N ** 3 / el, "decode_s": el,
           "decode_roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_TFLOPS["fp16"],
                               "unit": "TFLOP/s", "frac": ach / PEAK_TFLOPS["fp16"],
                               "flops_per_query": FLOPS_PER_QUERY_WIDEN,
                               "queries_per_launch": qpl, "avg_launch_ms": kms},
           "unet_sample_steps_per_s": sps, "unet_batch_per_rank": nl,
           "unet_path": "hipGraph of 1000 steps x 18 ldm_conv1d launches (direct staging)",
           "unet_conv_weight_bytes_per_step": wbytes}
    # roofline of the sampler step from its algorithmic work (unet.step_cost): the convs'
    # FLOPs against the fp32 MFMA peak (v_mfma_f32_16x16x4f32: fp32 activations, bf16 weights
    # widened) and their bytes against HBM; the larger of the two times is the bound.  Both
    # are far below the measured step: it is a chain of 18 dependent launches (DESIGN.md §9;
    # the launch-chain model of scripts/microbench/graph_chain_latency.hip is reported beside,
    # as a model, not as the roofline)
    cost = unet.step_cost(nl)
    t_mfma = cost["flops"] / (PEAK_TFLOPS["fp32"] * 1e12)
    t_hbm = cost["bytes"] / 8e12
    mf = t_mfma >= t_hbm
    res["unet_roofline"] = {
        "bound": "mfma" if mf else "hbm",
        "achieved": sps * (cost["flops"] / 1e12 if mf else cost["bytes"] / 1e9),
        "peak": PEAK_TFLOPS["fp32"] if mf else 8000.0, "unit": "TFLOP/s" if mf else "GB/s",
        "frac": sps * (t_mfma if mf else t_hbm),
        "flops_per_step": cost["flops"], "bytes_per_step": cost["bytes"],
        "hbm_frac": sps * t_hbm, "mfma_fp32_frac": sps * t_mfma,
        "note": "algorithmic FLOPs / bytes of the 18 convs of one step at this batch "
                "(UNet1DDenoiser.step_cost) x steps/s, against the fp32 MFMA peak the convs "
                "run on and HBM; the step is launch-chain-bound, far from either"}
    node = committed_graph_node_latency()
    if node is not None:
        res["unet_launch_chain_model"] = {
            "steps_per_s": 1.0 / (18 * node * 1e-9), "node_ns": node, "launches_per_step": 18,
            "frac": sps * 18 * node * 1e-9,
            "source": "profiles/r04a/graph_node_latency.json (scripts/microbench/"
                      "graph_chain_latency.hip, empty-kernel chain)",
            "note": "a MODEL (18 x one dependent graph node of empty kernels), not a roofline"}
    if rank == 0 and not args.no_cpu:
        res["unet_cpu_baseline"] = cpu_baseline_unet(min(5.0, args.cpu_seconds), nl)
    return res


def bench_decode_b1(args, rank, world, dev, group, decoder, desc, gen):
    """SURVEY §8(d) "B = 1 for the headline number": one shape's ``--grid``^3 decode (16.8 M
    queries at 256^3), z-slab over the ranks, ``--dtype``; kernel time from HIP events on its
    stream; §8(d)'s method: 3 warm-up and 10 timed decodes, the max-over-ranks wall time of the
    10 and the MEDIAN of the per-decode hipEvent times."""
    from ldm_sdf import ops
    N = args.grid
    lat1 = torch.randn(1, 256, device=dev, generator=gen) * 0.1
    out1 = torch.empty(1, N, N, N, device=dev)
    slab = SlabTimer(desc, lambda: ops.decoder_fold(desc, lat1), N,
                     torch.cuda.current_stream(dev))
    reps = 10
    ev = []
    el = run_decode_steps(slab, 1, N, steps=reps, warmup=3, world=world, group=group,
                          device=dev, out=out1, sync=torch.cuda.synchronize,
                          on_timed=lambda: setattr(slab, "timed", True), step_events=ev)
    kms, qpl = slab.kernel_stats()
    evs = event_summary(ev)
    ach = FLOPS_PER_QUERY * qpl / (kms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    return {"metric": f"SDF queries/sec, ONE shape on a {N}^3 grid", "value": N ** 3 * reps / el,
            "unit": "queries/s", "ms_per_decode": el / reps * 1e3, "dtype": args.dtype,
            "roofline": {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                         "frac": ach / peak, "kernel": "dec_fs_kernel",
                         "queries_per_launch": qpl, "avg_launch_ms": kms},
            "target_ms_at_40pct": N ** 3 * FLOPS_PER_QUERY / (0.4 * peak * 1e12) * 1e3,
            "step_time_events": evs,
            "value_from_median": N ** 3 / (evs["median_ms"] * 1e-3) if evs else None}


def committed_graph_node_latency():
    """The per-node latency of a dependent hipGraph chain of empty kernels, as measured by
    scripts/microbench/graph_chain_latency.hip (profiles/r04a/graph_node_latency.json, median
    over its grid sizes); None when absent."""
    f = os.path.join(ROOT, "profiles", "r04a", "graph_node_latency.json")
    try:
        rows = [json.loads(l) for l in open(f) if l.strip().startswith("{")]
        v = sorted(float(r["node_ns_median"]) for r in rows if "node_ns_median" in r)
    except (OSError, ValueError, KeyError):
        return None
    return v[len(v) // 2] if v else None


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: run this same command as N ranks under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) in a CHILD process --
    nothing here has touched the GPU -- and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def leg(name: str) -> None:
    """LDM_BENCH_TRACE=1: one stderr line per leg and rank, so a stalled multi-rank run shows
    where each rank is (with LDM_BENCH_WATCHDOG=<s>: every thread's stack after s seconds, then
    exit)."""
    if os.environ.get("LDM_BENCH_TRACE"):
        print(f"[bench rank {os.environ.get('RANK', '0')}] {name} "
              f"t={time.perf_counter() - _T0:.1f}s", file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if os.environ.get("LDM_BENCH_WATCHDOG"):
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["LDM_BENCH_WATCHDOG"]), exit=True)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
              f"torchrun --nproc-per-node {args.gpus} (or plain python, which spawns them)",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LDM_BENCH_BACKEND=gloo (a rehearsal of the multi-rank flow on a ONE-GPU box: every rank on
    # cuda:0, collectives over gloo -- RCCL refuses two ranks on one device); default: RCCL,
    # one GPU per rank
    backend = os.environ.get("LDM_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        # RCCL fails fast: an error / timeout on one rank aborts the communicator instead of
        # leaving the others blocked in a collective (SURVEY §5 "Fault/elastic")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if backend == "gloo":
            dist.init_process_group("gloo")
            # gloo's coalesced all-gather of DEVICE tensors never completed here (r06i: both
            # ranks waited on the group's handle for 150 s); the rehearsal takes the per-shape
            # form, which tests/test_dist_gloo.py pins bitwise to the coalesced one (RCCL runs
            # the coalesced form)
            from ldm_sdf.dist import set_gather_mode
            set_gather_mode("per_shape")
        else:
            dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD

    leg("process group up")
    import ldm_sdf
    from ldm_sdf import ops
    from ldm_sdf.dist import slab_bounds

    ldm_sdf.load_library()
    N, B = args.grid, args.batch
    decoder = ldm_sdf.SDFDecoder(256, seed=1234)
    gen = torch.Generator(device=dev).manual_seed(0)
    latents = torch.randn(B, 256, device=dev, generator=gen) * 0.1
    desc = decoder.device_pack(args.dtype, dev)["desc"]
    k0, k1, S = slab_bounds(rank, world, N)
    out = torch.empty(B, N, N, N, device=dev)
    stream = torch.cuda.current_stream(dev)
    slab = SlabTimer(desc, lambda: ops.decoder_fold(desc, latents), N, stream)
    spg = args.shapes_per_group or None
    local = []
    step_ev = []
    elapsed = run_decode_steps(slab, B, N, steps=args.steps, warmup=args.warmup, world=world,
                               group=group, device=dev, out=out, sync=torch.cuda.synchronize,
                               shapes_per_group=spg,
                               on_timed=lambda: setattr(slab, "timed", True), local=local,
                               step_events=step_ev)
    slab.timed = False
    leg("decode steps done")
    kms, qpl = slab.kernel_stats()
    multi = None
    if world > 1:
        # per rank: its step time, its slab kernels' time per step (HIP events) and the rest --
        # the part of the all-gathers the kernels did not hide -- plus the world the group saw
        multi = rank_breakdown(local[0] / args.steps * 1e3,
                               kms * len(slab.events) / max(1, args.steps), group, dev)
    total_q = B * N ** 3 * args.steps
    value = total_q / elapsed
    ach = FLOPS_PER_QUERY * qpl / (kms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    traffic, traffic_src = decoder_traffic(qpl)

    # SURVEY §8(d)'s single-shape headline: ONE shape's 256^3 grid (16.8 M queries), same kernel
    leg("rank breakdown done")
    b1 = bench_decode_b1(args, rank, world, dev, group, decoder, desc, gen)
    leg("decode_b1 done")

    res = None
    if rank == 0:
        res = {
            "metric": "SDF queries/sec on 256^3 grid (+ DDPM sample steps/sec)",
            "value": value, "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (latents N(0,0.1^2) seed 0, He-normal decoder seed 1234)",
            "config": {"workload": (f"config4: decode B={B} shapes on a {N}^3 grid, z-slab "
                                    f"sharded over {world} ranks + RCCL all-gathers of the "
                                    "volume (each group of ceil(B/8) shapes' per-shape gathers "
                                    "as one coalesced collective, overlapping the next group)")
                                   if world > 1 else
                                   (f"config4: decode B={B} shapes on a {N}^3 grid on 1 rank "
                                    "(the whole grid is the one slab: no gather)"),
                       "batch": B, "grid": N, "latent_dim": 256, "decoder": "DeepSDF 8x512 skip@4",
                       "parallelism": f"zslab{world}"},
            "roofline": {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                         "frac": ach / peak, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "dec_fs_kernel (+fs_aux_pack, <0.1%)",
                         "flops_per_query": FLOPS_PER_QUERY,
                         "queries_per_launch": qpl, "avg_launch_ms": kms,
                         "launches_per_step": len(slab.events) // max(1, args.steps)},
            "step_time_events": event_summary(step_ev),
            "decode_b1": b1,
        }
        if multi is not None:
            res["multi_gpu"] = multi
    if not args.no_ddpm:
        leg("ddpm")
        r = bench_ddpm(args, rank, world, dev, group, gen, decoder)
        if rank == 0:
            res["ddpm"] = r
    if rank == 0 and not args.no_mc:
        leg("mc")
        res["mc"] = bench_mc(out[0], args)
    if not args.no_config5:
        leg("config5")
        res_c5 = config5(args, rank, world, dev, group, gen)
        if rank == 0:
            res["config5"] = res_c5
    if rank == 0 and not args.no_train:
        leg("train")
        res["train"] = bench_train(args, dev, gen)
    if rank == 0 and not args.no_autodecoder:
        leg("autodecoder")
        res["autodecoder"] = bench_autodecoder(args, dev)
    if rank == 0 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_decode(N, args.cpu_seconds)
        if "ddpm" in res:
            res["ddpm"]["cpu_baseline"] = cpu_baseline_sampling(min(5.0, args.cpu_seconds),
                                                                args.ddpm_batch)
            if res["ddpm"].get("config3_sample_plus_decode128_s") is not None:
                # config 3 end to end on the CPU, from the two bounded samples just timed: 1000
                # oracle steps at B = 8 + the 8 x 128^3 decode at the oracle's q/s (flat in N)
                sps_c = res["ddpm"]["cpu_baseline"]["value"]
                qps_c = res["cpu_baseline"]["value"]
                e2e_c = 1000.0 / sps_c + args.ddpm_batch * 128 ** 3 / qps_c
                res["ddpm"]["config3_cpu_baseline"] = {
                    "value": e2e_c, "unit": "s (sample + decode, extrapolated)", "kind": "port",
                    "cores": res["cpu_baseline"]["cores"],
                    "sample": "1000 / ddpm.cpu_baseline steps/s + 8 x 128^3 / "
                              "cpu_baseline queries/s (both measured above on this host)",
                    "gpu_over_cpu": e2e_c / res["ddpm"]["config3_sample_plus_decode128_s"]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    leg("final barrier")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_ddpm(args, rank, world, dev, group, gen, decoder):
    """DDPM sampling, 1000 steps of ``--ddpm-batch`` latents, batch-sharded over the ranks
    (each rank samples its shard; steps/s = 1000 / max-over-ranks time), through the default
    ``Sampler`` path (the persistent one-launch loop) with the hipGraph per-step path timed
    beside it on the same inputs; then config 3 end to end (sample -> decode 128^3)."""
    import ldm_sdf
    den = ldm_sdf.MLPDenoiser(seed=4321)
    sch = ldm_sdf.DDPMSchedule()
    nb = args.ddpm_batch
    lo, hi = ldm_sdf.dist.batch_shard(nb, rank, world)
    nl = max(1, hi - lo)
    sampler = ldm_sdf.Sampler(den, sch, nl, dtype="bf16", device=dev)
    xT = torch.randn(nl, 256, device=dev, generator=gen)
    noise = torch.randn(1000, nl, 256, device=dev, generator=gen)
    sampler.run(xT, noise)            # first launch (module load) / capture
    reps = 3

    def timed(fn):
        if world > 1:
            dist.barrier(group)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        if world > 1:
            tt = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
            el = float(tt)
        return 1000 * reps / el

    # check=False (no host-side fallback inside the timed region), but the status word is read
    # after EVERY rep (it is re-zeroed per launch): a rep that stopped early would otherwise
    # shorten the time unseen.  One ~20 us read-back per 15-20 ms rep.
    persistent = sampler.loop is not None
    statuses = []

    def one_rep():
        sampler.run(xT, noise, check=False)
        if persistent:
            statuses.append(sampler.loop.status())
    sps = timed(one_rep)
    loop_status = max(statuses) if statuses else None
    loop_form = ldm_sdf.ops.sample_loop_last_form() if persistent else None
    sampler_g = ldm_sdf.Sampler(den, sch, nl, dtype="bf16", device=dev, persistent=False)
    xg = sampler_g.run(xT, noise).clone()
    sps_graph = timed(lambda: sampler_g.run(xT, noise))
    same = bool(torch.equal(sampler.run(xT, noise), xg))
    e2e, c3_dtype, c3 = None, None, {}
    # config 3 samples with the same random time MLP and residual blocks but identity in/out
    # projections (tests/test_gpu_ddpm.py bounded_denoiser_params): an untrained random
    # denoiser drives x to ~1e8 over 1000 steps, whose decode is meaningless (every 16-bit
    # dtype saturates); here the sampled latents stay O(1) (RMS ~0.45), the regime the 16-bit
    # decode is calibrated for.  The sampling work per step is the same network.
    den_c3 = bounded_denoiser(den)
    if not args.no_config3:      # config 3: sample(8) -> decode 128^3, end to end
        # the decoder's packed weights are a one-time setup (like loading the model): both
        # 16-bit packs exist before the clock starts, whichever dtype="auto" then picks
        for dt in ("bf16", "fp16"):
            decoder.device_pack(dt, dev)

        def clock():
            if world > 1:
                dist.barrier(group)
            torch.cuda.synchronize()
            return time.perf_counter()

        def e2e_call():
            lat_ = ldm_sdf.sample(den_c3, sch, nb, dtype="bf16", device=dev, group=group,
                                  generator=gen)
            dt_ = ldm_sdf.resolve_decode_dtype(args.dtype if args.dtype != "bf16" else "auto",
                                               lat_)
            ldm_sdf.decode(decoder, lat_, 128, dtype=dt_, group=group)
            return dt_

        # (1) the first API call of the process for this shape (fresh Sampler: its buffers,
        # loop program, first launches of the 128^3 decode) -- what one-shot use pays
        t2 = clock()
        c3_dtype = e2e_call()
        torch.cuda.synchronize()
        first = time.perf_counter() - t2
        # (2) the same API call again (fresh Sampler, warm process), 3 reps, median
        warm = []
        for _ in range(3):
            t2 = clock()
            e2e_call()
            torch.cuda.synchronize()
            warm.append(time.perf_counter() - t2)
        # (3) steady state: one Sampler kept across calls (no per-call setup), run + decode
        smp3 = ldm_sdf.Sampler(den_c3, sch, nl, dtype="bf16", device=dev)
        x3 = torch.randn(nl, 256, device=dev, generator=gen)
        n3 = torch.randn(1000, nl, 256, device=dev, generator=gen)
        smp3.run(x3, n3)
        steady = []
        for _ in range(3):
            t2 = clock()
            lat3 = smp3.run(x3, n3)
            lat3 = ldm_sdf.dist.all_gather_rows(lat3.clone(), nb, group=group) \
                if world > 1 else lat3
            ldm_sdf.decode(decoder, lat3, 128, dtype=c3_dtype, group=group)
            torch.cuda.synchronize()
            steady.append(time.perf_counter() - t2)
        warm.sort()
        steady.sort()
        e2e = warm[1]
        c3 = {"config3_first_call_s": first, "config3_api_call_s": warm,
              "config3_steady_s": steady, "config3_setup_s": warm[1] - steady[1],
              "config3_first_call_overhead_s": first - warm[1]}
    wbytes = 2 * (den.H * den.D * 2 + den.n_blocks * den.H * den.H) + 2 * nl * den.D * 4
    valid = not loop_status
    hand = handoff_latency()
    if hand is not None:
        # latency model: each reverse step is 6 dependent layer hand-offs (in-projection, 4
        # blocks, out-projection + update), each at least one same-XCD publish -> poll latency
        model_step = 6 * hand["one_way_ns"] * 1e-9
        roof = {"bound": "handoff-latency", "achieved": sps,
                "peak": 1.0 / model_step, "unit": "steps/s", "frac": sps * model_step,
                "handoffs_per_step": 6, "one_way_handoff_ns": hand["one_way_ns"],
                "source": hand["source"],
                "note": "peak = 1 / (6 x measured same-XCD 8-byte tagged hand-off latency); "
                        "frac = that model step time / the measured step time"}
    else:
        roof = None
    ag = allgather_latency()
    roof_ag = None
    if ag is not None:
        # each layer boundary is in fact an all-gather of the layer inside the XCD replica
        # (32 workgroups publish 32 rows each, every one stages all 1024): 6 per step
        model_ag = 6 * ag["phase_ns"] * 1e-9
        roof_ag = {"bound": "xcd-allgather-latency", "achieved": sps, "peak": 1.0 / model_ag,
                   "unit": "steps/s", "frac": sps * model_ag, "allgathers_per_step": 6,
                   "allgather_phase_ns": ag["phase_ns"], "source": ag["source"],
                   "note": "peak = 1 / (6 x the measured per-layer all-gather of 1024 tagged "
                           "granules among 32 workgroups of one XCD, no arithmetic)"}
    return {"metric": "DDPM sample steps/sec", "value": sps if valid else None,
            "valid": valid, "unit": "steps/s",
            "batch": nb, "batch_per_rank": nl, "T": 1000, "shape_steps_per_s": sps * nb,
            "path": (({"replica": "one persistent launch for all 1000 steps: one network "
                                  "copy per XCD in registers, XCD-local tagged hand-offs "
                                  "per layer (sample_replica_kernel)",
                       "chipwide": "one persistent launch for all 1000 steps: weights in "
                                   "registers, XCD-hierarchical grid barrier per layer"}
                      .get(loop_form, f"persistent loop ({loop_form})")) if persistent
                     else "hipGraph of 1000 fused steps (6 kernels each)"),
            "loop_status": loop_status, "loop_status_per_rep": statuses,
            "loop_form": loop_form,
            "graph_path": {"steps_per_s": sps_graph,
                           "path": "hipGraph of 1000 fused steps (6 kernels each)",
                           "bit_identical": same},
            "roofline": roof,
            "roofline_allgather": roof_ag,
            "roofline_hbm": {"bound": "hbm", "achieved": sps * wbytes / 1e9,
                         "peak": 8000.0, "unit": "GB/s",
                         "frac": sps * wbytes / 8e12,
                         "bytes_per_step": wbytes,
                         "note": "SURVEY §8(d) bytes: weights streamed once per "
                                 "step + x, eps; the persistent loop holds weights "
                                 "in registers, so it is grid-barrier-latency-bound "
                                 "(DESIGN.md §5)"},
            "config3_sample_plus_decode128_s": e2e,
            "config3": (f"sample(8) (1000 bf16 steps) -> decode(128^3, {c3_dtype}: dtype='auto' "
                        f"for these latents, api.resolve_decode_dtype), wall time; "
                        f"config3_sample_plus_decode128_s = median of 3 API calls in a warm "
                        f"process (each builds a fresh Sampler); config3_steady_s = one Sampler "
                        f"reused (run + decode); config3_first_call_s = the process's first "
                        f"call (first launches of the 128^3 decode and the loop)"
                        if e2e is not None else None),
            "config3_decode_dtype": c3_dtype if e2e is not None else None, **c3}


def bounded_denoiser(den):
    """``den`` with identity in/out projections (W_in = [I; 0], W_out = [I, 0], zero in/out
    biases) and its blocks and time MLP unchanged: every reverse step contracts, so sampled
    latents stay O(1) (tests/test_gpu_ddpm.py bounded_denoiser_params)."""
    import ldm_sdf
    p = {k: v.detach().cpu().clone() for k, v in den.params.items()}
    D, H = den.D, den.H
    p["Win"] = torch.zeros(H, D)
    p["Win"][:D] = torch.eye(D)
    p["Wout"] = torch.zeros(D, H)
    p["Wout"][:, :D] = torch.eye(D)
    p["bin"] = torch.zeros(H)
    p["bout"] = torch.zeros(D)
    return ldm_sdf.MLPDenoiser(D=D, H=H, n_blocks=den.n_blocks, TE=den.TE, T=den.T, params=p)


def bench_train(args, dev, gen):
    """Config 2: DDPM training on 1k synthetic 256-d latents, MLP denoiser, bf16, batch 1000."""
    import ldm_sdf
    den_t = ldm_sdf.MLPDenoiser(seed=4321)
    sch_t = ldm_sdf.DDPMSchedule()
    lat_t = torch.randn(1000, 256, device=dev, generator=gen) * 0.5
    # (group=LOCAL: config 2 is a 1-GPU workload; at world > 1 only rank 0 runs this leg, so
    # train() must not enter a collective the other ranks never join)
    from ldm_sdf.dist import LOCAL
    st = ldm_sdf.train(den_t, sch_t, lat_t, steps=3, batch=1000, dtype="bf16",
                       group=LOCAL)   # warm-up
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    st = ldm_sdf.train(den_t, sch_t, lat_t, steps=args.train_steps, batch=1000,
                       dtype="bf16", state=st, group=LOCAL)
    torch.cuda.synchronize()
    dtt = (time.perf_counter() - t3) / args.train_steps
    H, D, nb = den_t.H, den_t.D, den_t.n_blocks
    macs = 1000 * (H * 128 + H * H + H * D + nb * H * 2 * H + D * H)   # forward MACs
    flops = 3 * 2 * macs          # forward + the two backward products (dX, dW) per layer
    ach = flops / dtt / 1e12
    res = {"metric": "DDPM training steps/sec (config 2)", "value": 1.0 / dtt,
           "unit": "steps/s", "batch": 1000, "ms_per_step": dtt * 1e3,
           "tflops_fwd_bwd": ach,
           "roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_TFLOPS["bf16"],
                        "unit": "TFLOP/s", "frac": ach / PEAK_TFLOPS["bf16"],
                        "flops_per_step": flops,
                        "note": "3 x 2 x forward MACs per step (1000 samples) over the wall "
                                "time of a step (every launch incl. AdamW, 100 timed steps)"},
           "loss_first_last": [st.losses[0], st.losses[-1]]}
    res["form"] = ldm_sdf.ops.train_step_last_form()
    # the other form of the same step, same model state, for the record:
    # the one-launch DAG step when "auto" ran the launches, and the other way round
    from ldm_sdf import ops as _ops
    other = "dag" if res["form"] == "launches" else "launches"
    try:
        _ops.train_step_config(other)
        st = ldm_sdf.train(den_t, sch_t, lat_t, steps=3, batch=1000, dtype="bf16", state=st,
                           group=LOCAL)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        st = ldm_sdf.train(den_t, sch_t, lat_t, steps=args.train_steps, batch=1000,
                           dtype="bf16", state=st, group=LOCAL)
        torch.cuda.synchronize()
        d_o = (time.perf_counter() - t4) / args.train_steps
        res["other_form"] = {"form": _ops.train_step_last_form(), "steps_per_s": 1.0 / d_o,
                             "ms_per_step": d_o * 1e3,
                             "note": "same step, bit-identical results (tests/test_gpu_train_dag.py); "
                                     "value is the form 'auto' picks"}
    finally:
        _ops.train_step_config("auto")
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_train(min(10.0, args.cpu_seconds))
    return res


if __name__ == "__main__":
    main()
