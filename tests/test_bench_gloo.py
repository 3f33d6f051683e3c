"""bench.py's multi-rank path without a GPU: the per-rank step loop (``run_decode_steps``: warm-up,
barrier + sync brackets, max-over-ranks time) driving ``dist.decode_sharded`` over gloo at
world size 2, with a synthetic exact slab function and the oracle decoder as the slab
function.  The assembled volumes must equal the world-1 run bit for bit.  Also: the
``--gpus`` / WORLD_SIZE consistency check exits before anything touches a GPU."""
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from tests.test_dist_gloo import _run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _exact_slab(N):
    def slab(k0, k1, dst, b0, b1):
        b = torch.arange(b0, b1).view(-1, 1, 1, 1).float()
        k = torch.arange(k0, k1).view(1, -1, 1, 1).float()
        j = torch.arange(N).view(1, 1, N, 1).float()
        i = torch.arange(N).view(1, 1, 1, N).float()
        dst.copy_(b * 1e6 + k * 1e4 + j * 100 + i)
    return slab


def _oracle_slab(N, calls):
    from oracle import ref_cpu as R
    p = R.make_decoder_params(L=16, H=64, seed=2)
    z = torch.randn(5, 16, generator=torch.Generator().manual_seed(0), dtype=torch.float64)

    def slab(k0, k1, dst, b0, b1):
        calls.append((k0, k1, b0, b1))
        dst.copy_(R.decode_grid(p, z[b0:b1], N, k0, k1).float())
    return slab


def _bench_steps(rank, world):
    sys.path.insert(0, ROOT)
    import bench
    out = {}
    for name, B, N, spg in (("exact", 4, 12, None), ("exact_uneven", 3, 11, 2),
                            ("oracle", 5, 8, 2)):
        calls = []
        slab = _oracle_slab(N, calls) if name == "oracle" else _exact_slab(N)
        vol = torch.empty(B, N, N, N)
        loc = []
        el = bench.run_decode_steps(slab, B, N, steps=2, warmup=1, world=world, group=None,
                                    device=torch.device("cpu"), out=vol, shapes_per_group=spg,
                                    local=loc)
        assert len(loc) == 1 and 0 < loc[0] <= el
        # the same on this rank alone (world 1): the reference volume
        ref = torch.empty(B, N, N, N)
        bench.run_decode_steps(slab, B, N, steps=1, warmup=0, world=1, group=None,
                               device=torch.device("cpu"), out=ref)
        # max over ranks: every rank reports the same elapsed
        t = torch.tensor([el], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        out[name] = (bool(torch.equal(vol, ref)), float(t) == float(mx), el > 0)
    # the per-rank breakdown the bench reports at world > 1
    br = bench.rank_breakdown(10.0 + rank, 4.0, None, torch.device("cpu"))
    ok = (br["world_seen"] == world and br["backend"] == "gloo" and
          [p["rank"] for p in br["per_rank"]] == list(range(world)) and
          all(p["gather_exposed_ms"] == 6.0 + p["rank"] for p in br["per_rank"]))
    out["breakdown"] = (ok, True, True)
    return out


def test_bench_decode_steps_world2_equals_world1():
    res = _run("tests.test_bench_gloo:_bench_steps", 2)
    for r in range(2):
        assert isinstance(res[r], dict), res[r]
        for name, (same, maxed, pos) in res[r].items():
            assert same and maxed and pos, (r, name, res[r][name])


@pytest.mark.parametrize("env_world,gpus", [("2", 4), ("4", 1)])
def test_bench_rejects_world_mismatch(env_world, gpus):
    """WORLD_SIZE from a launcher that disagrees with --gpus: exit 2 before any GPU call."""
    env = dict(os.environ, WORLD_SIZE=env_world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE" in r.stderr
