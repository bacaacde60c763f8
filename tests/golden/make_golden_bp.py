"""Golden vectors for the QSGDBP call site (compressors.py:324-378, the
bit-packed QSGD compressor whose packing runs in the reference's C++
extension).  Run in the build container only:

    python tests/golden/make_golden_bp.py      -> tests/golden/qsgdbp.npz

The reference keeps QSGDBPCompressor commented out (it needs the custom
extension), so the vectors are produced from the reference's LIVE pieces:
  * xi: |QSGDMaxNormCompressor.compress(norm, x)| of the imported
    compressors.py — the same arithmetic and the same single bernoulli over n
    elements as the commented compress (compressors.py:346-353 = 302-312), so
    under torch.manual_seed the draws are identical; norm is the bucket's own
    max (compressors.py:341);
  * sign bit: 1 iff x < 0 (compressors.py:344-346: sign * -1, then -1 -> 0);
  * packed words: bitpacking.packing / unpacking of the reference's own C++
    extension compiled from its sources (oracle/build_ref.py), on int32 input;
  * decompress: unpack, [:n], {1 -> -1, 0 -> +1}, (norm / s) * sign * xi
    (compressors.py:369-378).
Data only (npz, no pickles); no reference source is copied.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import compressors  # noqa: E402  (reference)
from make_golden import edge_input  # noqa: E402

from oracle import build_ref  # noqa: E402

SEED = 42
CPU = torch.device("cpu")


def case(x: np.ndarray, bits: int, bitpacking):
    n = x.size
    s = (1 << bits) - 1
    t = torch.from_numpy(x.copy())
    norm = t.abs().max()
    torch.manual_seed(SEED)
    q = compressors.QSGDMaxNormCompressor(CPU, bits).compress(norm, t)
    xi = q.to(torch.int32).abs()
    sign = (t < 0).to(torch.int32)
    sign_packed = bitpacking.packing(sign)
    xi_packed = bitpacking.packing(xi)
    c = norm / s
    su = bitpacking.unpacking(sign_packed)[:n].clone()
    xu = bitpacking.unpacking(xi_packed)[:n]
    su[su == 1] = -1
    su[su == 0] = 1
    dec = c * su * xu
    return dict(x=x, bits=np.int32(bits), seed=np.int64(SEED), norm_over_s=np.float32(c.item()),
                sign_packed=sign_packed.numpy().astype(np.int32), xi_packed=xi_packed.numpy().astype(np.int32),
                xi_size=np.int64(xi_packed.numel()), dec=dec.numpy().astype(np.float32))


def main():
    bitpacking, _ = build_ref.load()
    out = {}
    for bits in (2, 4, 8):
        for n in (1, 37, 4099, 30_011):
            x = edge_input(n, seed=1000 * bits + n)
            for k, v in case(x, bits, bitpacking).items():
                out[f"b{bits}_n{n}/{k}"] = v
    path = os.path.join(HERE, "qsgdbp.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    main()
