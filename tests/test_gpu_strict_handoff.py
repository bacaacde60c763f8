"""The in-launch hand-offs built both ways agree.

The default build hands the absmax block partials and the greedy4 pack's
tile tables between workgroups with sc1 (write-through) stores and loads and
no fences — a gfx950 hardware property (MI355X_MICROARCH.md, the sc1 hand-off
table), not the HIP memory model.  `make strict` builds the memory model's
own release / acquire form (GC_STRICT_HANDOFF=1 -> lib/libgcodec_strict.so).
Here the strict library runs in a child process on the same inputs and its
max-norms and packed words must equal the default library's bit for bit."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRICT = os.path.join(ROOT, "gradient-compression_amd", "lib", "libgcodec_strict.so")

CHILD = r'''
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch, gcodec
from gcodec import codec, _lib
dev = torch.device("cuda", 0)
out = {"lib": _lib.LIB_PATH}
for n in (1, 4099, 1_000_003, 23_520_842, 100_000_000):
    g = torch.Generator(device=dev).manual_seed(n % 97)
    x = torch.randn(n, device=dev, generator=g).mul_(0.01)
    out[f"absmax_{n}"] = [float(codec.absmax(x).item()) for _ in range(3)]
    if n in (1_000_003, 23_520_842):
        v = torch.randint(0, 16, (n,), device=dev, generator=g, dtype=torch.int32)
        v[::97] = 200
        pk = codec.Greedy4Device(n, dev)
        hs = []
        for _ in range(3):
            pk.pack(v)
            w = pk.words[:pk.result()].cpu().numpy()
            hs.append(hashlib.sha256(w.tobytes()).hexdigest())
        out[f"g4_{n}"] = hs
print(json.dumps(out))
'''


def _run(lib):
    env = dict(os.environ)
    if lib:
        env["GCODEC_LIB"] = lib
    else:
        env.pop("GCODEC_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "gradient-compression_amd")], env=env,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_strict_release_acquire_build_equals_default():
    if not os.path.exists(STRICT):
        pytest.fail(f"{STRICT} not built (make -C gradient-compression_amd/csrc strict)")
    a, b = _run(None), _run(STRICT)
    assert a["lib"] != b["lib"] and b["lib"].endswith("libgcodec_strict.so")
    keys = [k for k in a if k != "lib"]
    assert keys and all(a[k] == b[k] for k in keys), {k: (a[k], b[k]) for k in keys if a[k] != b[k]}
    for k in keys:  # and each is stable call to call
        assert len(set(map(str, a[k]))) == 1, (k, a[k])
