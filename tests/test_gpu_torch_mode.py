"""Torch-mode draws (the reference's MT19937 stream, compressors.py:310 under
seed.py:6-11) generated on the GPU side stream with the next same-size call
generated speculatively (codec.mt19937_draws, MT_SPECULATE): every call must
return exactly torch's next `count` draws and leave torch's CPU generator
where torch.bernoulli would — across repeated sizes (speculation used),
changed sizes (speculation dropped), torch's generator used or reseeded in
between (speculation invalid), and with speculation off.  The oracle is the
serial MT19937 of oracle/gcodec_oracle.c continued from torch's state."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

import gcodec  # noqa: E402
from gcodec import codec  # noqa: E402
from gcodec.rng import torch_mt_state  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)


def _oracle_next(count):
    """(draws, state words, read index) of torch's generator after `count` more draws"""
    words, idx = torch_mt_state()
    st = O.MT19937(0)
    st._st.s[:] = [int(v) for v in words]
    st._st.idx = idx
    d = st.draws(count)
    w2, i2 = st.state()
    return d, np.asarray(w2, dtype=np.uint32), int(i2)


@pytest.mark.parametrize("speculate", [True, False])
def test_draw_sequences_vs_serial_stream(speculate):
    old = codec.MT_SPECULATE
    codec.MT_SPECULATE = speculate
    try:
        torch.manual_seed(123)
        seq = [300_007, 300_007, 300_007, 5_000, 5_000, 624, 1, 300_007, 300_007, 2 * 300_007]
        for i, cnt in enumerate(seq):
            ref, w2, i2 = _oracle_next(cnt)
            got = codec.mt19937_draws(cnt, DEV)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), ref), (i, cnt)
            words, idx = torch_mt_state()
            assert idx == i2 and np.array_equal(words, w2), (i, cnt)
            if i == 4:
                torch.rand(7)  # torch's generator used between two calls
            if i == 6:
                torch.manual_seed(99)  # and reseeded
    finally:
        codec.MT_SPECULATE = old


def test_torch_mode_compressor_back_to_back_vs_oracle():
    """QSGDMaxNormCompressor.compress in torch mode, five back-to-back calls on
    the same bucket (the speculative draws used four times), then the fused
    generator-quantize path in between (its own state buffers): q == the
    oracle's quantize of the serial stream every time."""
    n, bits = 1_000_003, 4
    x = O.gen_input(n, seed=3)
    xd = torch.from_numpy(x).to(DEV)
    norm = O.absmax(x)
    gcodec.set_rng_mode("torch")
    try:
        torch.manual_seed(5)
        c = gcodec.QSGDMaxNormCompressor(DEV, bits)
        for i in range(6):
            ref_draws, _, _ = _oracle_next(n)
            if i == 3:
                q = codec.qsgd_quantize_torch(xd, float(norm), bits)
            else:
                q = c.compress(torch.tensor([norm], device=DEV), xd)
            exp = O.qsgd_quantize(x, norm, bits, O.stream_rng(ref_draws))
            assert np.array_equal(q.cpu().numpy().astype(np.int32), np.asarray(exp, dtype=np.int32)), i
    finally:
        gcodec.set_rng_mode("philox")
