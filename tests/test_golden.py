"""The committed fixtures (tests/golden/*.npz) are the oracle's outputs: re-derive every case
on the CPU and compare, so the oracle and the vectors the GPU box checks against cannot
drift apart (tests/golden/make_golden.py is the generator)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as MG  # noqa: E402


@pytest.mark.parametrize("name", sorted(MG.CASES))
def test_golden_fixture_rederives(name):
    path = os.path.join(HERE, "golden", f"{name}.npz")
    have = dict(np.load(path))
    want = MG.CASES[name]()
    assert set(have) == set(want), name
    for k, v in want.items():
        v = np.asarray(v)
        assert have[k].shape == v.shape and have[k].dtype == v.dtype, (name, k)
        if v.dtype.kind in "iub":
            np.testing.assert_array_equal(have[k], v, err_msg=f"{name}.{k}")
        else:
            np.testing.assert_allclose(have[k], v, rtol=1e-9, atol=1e-12, err_msg=f"{name}.{k}")
