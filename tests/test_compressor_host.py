"""Host logic of the packed multi-scale compressors (no GPU): which backend
calls encode_mask / encode make for each world size and q_cache setting.  A
recording stand-in backend replaces the HIP codec; only the call pattern is
checked here (the words themselves are checked on the GPU against the oracle)."""
import pytest
import torch

import gcodec


class _Rec:
    """Records ms_* calls; ms_cache_bytes says 1 byte per element."""

    def __init__(self, cache_bytes=1):
        self.calls = []
        self.cache_bytes = cache_bytes

    def ms_cache_bytes(self, n, levels):
        return self.cache_bytes

    def ms_mask_encode(self, x, norm, levels, rng, world=1, idx=None, cache=None):
        self.calls.append(("mask", world, cache is not None))
        return torch.zeros(4, dtype=torch.int32)

    def ms_select_encode(self, x, norm, levels, rng, mask_words, world=1, idx=None, cache=None):
        self.calls.append(("select", world, cache is not None))
        return torch.zeros(4, dtype=torch.int32)

    def mt19937_draws(self, count, device):  # torch-mode reservations (unused here)
        raise AssertionError("philox only")


@pytest.mark.parametrize("q_cache,world,cached", [(None, 1, False), (None, 2, True), (None, 8, True),
                                                  (True, 1, True), (False, 4, False)])
@pytest.mark.parametrize("cls,kw", [(gcodec.QSGDMaxNormTwoScaleCompressor, dict(lower_quantization_level=2,
                                                                               higher_quantization_level=4)),
                                    (gcodec.QSGDMaxNormMultiScaleCompressor, dict(quantization_levels=[2, 4, 6]))])
def test_q_cache_default_follows_world_size(cls, kw, q_cache, world, cached):
    rec = _Rec()
    c = cls("cpu", generator=gcodec.Generator(1, "philox"), q_cache=q_cache, **kw)
    c.backend = rec
    x = torch.zeros(64, dtype=torch.float32)  # 16-byte aligned allocation
    m = c.encode_mask(torch.ones(1), x, world)
    c.encode(torch.ones(1), x, m, world)
    assert rec.calls == [("mask", world, cached), ("select", world, cached)]


def test_q_cache_needs_a_cache_form():
    """levels without a cache form (ms_cache_bytes == 0) run the two passes
    without one even at W > 1."""
    rec = _Rec(cache_bytes=0)
    c = gcodec.QSGDMaxNormTwoScaleCompressor("cpu", 9, 10, generator=gcodec.Generator(1, "philox"))
    c.backend = rec
    x = torch.zeros(64, dtype=torch.float32)
    c.encode(torch.ones(1), x, c.encode_mask(torch.ones(1), x, 4), 4)
    assert rec.calls == [("mask", 4, False), ("select", 4, False)]
