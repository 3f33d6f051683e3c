"""The C ABI's error behaviour from C (tests/c/abi_errors.c): every entry point of
include/ldm_sdf.h called with invalid arguments returns an error code and leaves a message in
ldm_last_error(); the host-only entry points (ABI version, workspace sizes, AdamW scalars, the
marching-cubes table, the one-launch training step's job table built from descriptors) work
without a GPU.  Here the checker is built with gcc against the product library; the same source
runs under host AddressSanitizer with `make -C latent-diffusion-models-for-shape-sdfs_amd/csrc
check-asan` (libldm_sdf_asan.so; log under profiles/)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd", "ldm_sdf")


def test_abi_errors_from_c(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libldm_sdf.so")):
        pytest.fail("libldm_sdf.so is not built (make -C .../csrc)")
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "abi_errors")
    subprocess.run([cc, "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_errors.c"), "-o", exe, "-L", LIBDIR,
                    "-lldm_sdf", "-Wl,-rpath," + LIBDIR], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
