"""Worker of tests/test_gpu_rccl.py: ONE rank on cuda:0 with the ``nccl`` backend (RCCL on
ROCm), so the package's collectives run through RCCL itself on the MI355X.  World 1 is all a
one-GPU box allows (RCCL refuses two ranks on one device); the calls below do not shortcut at
world 1 (the package's helpers that would are called at their collective level).  Writes a JSON
record to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    from ldm_sdf import dist as ld
    ld.init_process_group("nccl", device_id=dev)
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    g = torch.Generator(device=dev).manual_seed(1)
    B, N = 5, 32
    local = torch.randn(B, N, N, N, device=dev, generator=g)
    ok = {}
    for mode in ("coalesced", "per_shape"):
        ld.set_gather_mode(mode)
        dsts = [(b, torch.full((N, N, N), float("nan"), device=dev)) for b in range(B)]
        h = ld._gather_group(dsts, local, dist.group.WORLD)
        h.wait()
        torch.cuda.synchronize()
        ok[mode] = all(torch.equal(d, local[b]) for b, d in dsts)
        rec[f"mode_after_{mode}"] = ld.gather_mode()
    rec["gather_exact"] = ok
    # the flat gradient buffer's in-place all-reduce (what _allreduce_ issues at world > 1)
    flat, views = ld.flat_buffers({"a": (7, 3), "b": (5,)}, dev)
    flat.copy_(torch.arange(flat.numel(), device=dev, dtype=torch.float32))
    want = flat.clone()
    dist.all_reduce(flat)
    torch.cuda.synchronize()
    rec["allreduce_exact"] = bool(torch.equal(flat, want))
    # bench.py's per-rank breakdown (an all_gather of device tensors)
    sys.path.insert(0, ROOT)
    import bench
    rec["breakdown"] = bench.rank_breakdown(12.5, 10.0, dist.group.WORLD, dev)
    dist.barrier()
    dist.destroy_process_group()
    with open(sys.argv[1], "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()
