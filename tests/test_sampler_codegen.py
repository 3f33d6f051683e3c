"""The XCD-replica sampling loop's code generation (csrc/sample_loop.hip),
checked on the CPU from the compiler's own assembly of the product flags.

Round 5's fast sampler depended on a build accident: the loop's weights overflowed the 256
VGPRs a wave has at two waves per SIMD, the compiler spilled residual-block weight vectors to
scratch and reloaded them SERIALLY every step (scratch_load + s_waitcnt vmcnt(0), 5-6 times),
and the diagnostic stamps merely changed which values spilled.  Round 6 keeps the last residual
block's weights in LDS (SL_LDSBLK), which leaves the kernel without any scratch; and what the
stamps really bought -- the wave pausing right after a layer's publish before it polls for the
next layer -- is now built on purpose (SL_PUBFENCE: a scheduling barrier + s_sleep SL_PUBSLEEP,
4 after the round-6 sweep).  This test fails if a change (or a compiler update) brings the
spills back to the bench's configuration (D = 256, B <= 8: sample_replica_kernel<256, 1>), with
or without the stamps, or separates a publish from its pause."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _asm(tmp_path, *defines):
    if not os.path.exists(HIPCC) or shutil.which("make") is None:
        pytest.skip("hipcc not available")
    out = str(tmp_path / "sample_loop.s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
           "--cuda-device-only", "-S", *defines, os.path.join(CSRC, "sample_loop.hip"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return open(out).read()


def _kernel_stats(s, d, mbx):
    name = [n for n in re.findall(r"^(_ZN3ldm\w+sample_replica_kernel\w+):", s, re.M)
            if f"ILi{d}ELi{mbx}E" in n]
    assert len(name) == 1, name
    n = name[0]
    body = s[s.index(n + ":"):s.index(".Lfunc_end", s.index(n + ":"))]
    priv = int(re.search(re.escape(n) + r"\.private_seg_size, (\d+)", s).group(1))
    return priv, len(re.findall(r"\bscratch_(load|store)", body))


@pytest.mark.parametrize("stamp", [0, 1])
def test_replica_loop_has_no_scratch(tmp_path, stamp):
    """sample_replica_kernel<256, 1> (config 3 / the bench: D = 256, B = 8) builds with no
    scratch at all -- product flags, and with the diagnostic stamps too."""
    s = _asm(tmp_path, f"-DSL_STAMP={stamp}")
    priv, nscr = _kernel_stats(s, 256, 1)
    assert priv == 0 and nscr == 0, (priv, nscr)


def test_every_publish_is_followed_by_its_pause(tmp_path):
    """The six tagged publishes of a step (8-byte agent-scope stores: global_store_dwordx2 ...
    sc1) each have the s_sleep of after_publish() within the next few instructions."""
    s = _asm(tmp_path)
    n = [x for x in re.findall(r"^(_ZN3ldm\w+sample_replica_kernel\w+):", s, re.M)
         if "ILi256ELi1E" in x][0]
    body = s[s.index(n + ":"):s.index(".Lfunc_end", s.index(n + ":"))]
    ins = [l.strip() for l in body.split("\n") if l.strip() and not l.strip().startswith((";", "."))]
    pubs = [k for k, l in enumerate(ins) if l.startswith("global_store_dwordx2") and "sc1" in l]
    assert len(pubs) >= 6, len(pubs)
    for k in pubs:
        assert any(l.startswith("s_sleep") for l in ins[k + 1:k + 13]), ins[k:k + 13]
