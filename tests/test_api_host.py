"""Host-side logic of the Python API that needs no GPU: the dtype="auto" cache of
``resolve_decode_dtype`` cannot hand a freed tensor's decision to a new tensor."""
import torch


def test_auto_cache_does_not_match_a_new_tensor_at_a_reused_id():
    """A new latents tensor that lands on a freed one's id, storage and version (CPython and the
    caching allocator both reuse) must get its own RMS decision: small-RMS latents resolve to
    bf16, then large-RMS latents at the SAME cache key resolve to fp32, not the cached bf16."""
    from ldm_sdf import api
    api.clear_auto_cache()
    small = torch.randn(4, 256, generator=torch.Generator().manual_seed(0)) * 0.05
    assert api.resolve_decode_dtype("auto", small) == "bf16"
    big = torch.randn(4, 256, generator=torch.Generator().manual_seed(1)) * 3.0
    # force the collision: the small tensor's entry moved under the big one's id, with the big
    # one's (data_ptr, version, shape, device) -- everything the round-5 key compared
    ref, _, pick = api._AUTO_CACHE.pop(id(small))
    api._AUTO_CACHE[id(big)] = (ref, (big.data_ptr(), big._version, tuple(big.shape),
                                      str(big.device)), pick)
    assert api.resolve_decode_dtype("auto", big) == "fp32"
    # a genuine repeat of the same unmodified tensor is a hit (no second RMS read needed)
    assert api._AUTO_CACHE[id(big)][0]() is big
    assert api.resolve_decode_dtype("auto", big) == "fp32"
    # an in-place write bumps the version: re-decided
    big.mul_(0.01)
    assert api.resolve_decode_dtype("auto", big) == "bf16"


def test_auto_cache_thresholds():
    from ldm_sdf import api
    api.clear_auto_cache()
    z = torch.ones(2, 256)
    for scale, want in ((0.1, "bf16"), (0.5, "fp16"), (2.0, "fp32")):
        assert api.resolve_decode_dtype("auto", z * scale) == want
    assert api.resolve_decode_dtype("fp16", z * 9.0) == "fp16"
