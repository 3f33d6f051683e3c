"""The package's collectives through RCCL itself on the MI355X (every
multi-rank test so far ran gloo).  One rank with the ``nccl`` backend (= RCCL on ROCm) -- a
one-GPU box allows no more: RCCL refuses two ranks on one device -- launched as a child
``torch.distributed.run``: the z-slab decode's grouped gather in both forms (the coalesced one
must be accepted by RCCL's coalescing manager, not fall back), the flat gradient buffer's
in-place all-reduce and the bench's per-rank breakdown, all exact."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_collectives_exact(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path / "rccl.json")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.join(ROOT, "tests", "rccl_worker.py"), out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rec = json.load(open(out))
    print(rec)
    assert rec["backend"] == "nccl" and rec["world"] == 1
    assert rec["gather_exact"] == {"coalesced": True, "per_shape": True}
    assert rec["mode_after_coalesced"] == "coalesced"       # RCCL took the coalescing manager
    assert rec["allreduce_exact"]
    b = rec["breakdown"]
    assert b["world_seen"] == 1 and b["backend"] == "nccl"
    assert b["per_rank"][0]["gather_exposed_ms"] == pytest.approx(2.5)
