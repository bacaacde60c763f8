"""Build the reference's own C++ packing extensions from their sources, in
place under /root/reference, into oracle/_ref/ (git-ignored; travels to the GPU
box with the snapshot).  TEST INFRASTRUCTURE ONLY.

Sources (read-only, never copied):
  /root/reference/extensions/Extension CPU/bitpacking.cpp        -> _ref/bitpacking/bitpacking.so
  /root/reference/extensions/Extension CPU BP/bytepacking.cpp    -> _ref/bytepacking/bytepacking.so
  /root/reference/extensions/Extension GPU/gpu_bitpacking.cpp    -> _ref/gpu_bitpacking/gpu_bitpacking.so

They are plain ATen/pybind11 CppExtensions (setup.py:10-14 in each directory);
they compile against the image's own torch headers with g++ via
torch.utils.cpp_extension — no stand-in headers, no reference build system.

    python oracle/build_ref.py          # build (needs /root/reference)
    build_ref.load()                    # import the prebuilt modules
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")
REF_EXT = "/root/reference/extensions"
SOURCES = {
    "bitpacking": os.path.join(REF_EXT, "Extension CPU", "bitpacking.cpp"),
    "bytepacking": os.path.join(REF_EXT, "Extension CPU BP", "bytepacking.cpp"),
    "gpu_bitpacking": os.path.join(REF_EXT, "Extension GPU", "gpu_bitpacking.cpp"),
}


def _so(name: str) -> str:
    return os.path.join(OUT, name, f"{name}.so")


def build(verbose: bool = False) -> bool:
    """Compile the reference extensions if /root/reference is present."""
    if not all(os.path.exists(p) for p in SOURCES.values()):
        return False
    import torch  # noqa: F401
    from torch.utils.cpp_extension import load

    for name, src in SOURCES.items():
        if os.path.exists(_so(name)) and os.path.getmtime(_so(name)) >= os.path.getmtime(src):
            continue
        bdir = os.path.join(OUT, name)
        os.makedirs(bdir, exist_ok=True)
        load(name=name, sources=[src], build_directory=bdir, verbose=verbose,
             extra_cflags=["-O2"])
    return True


def available() -> bool:
    return all(os.path.exists(_so(n)) for n in ("bitpacking", "bytepacking"))


def _import(name: str):
    import torch  # noqa: F401  (the extension links libtorch)

    spec = importlib.util.spec_from_file_location(name, _so(name),
                                                  loader=importlib.machinery.ExtensionFileLoader(name, _so(name)))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load():
    """(bitpacking, bytepacking) modules from oracle/_ref (builds if needed)."""
    if not available():
        if not build():
            raise RuntimeError("oracle/_ref not built and /root/reference absent")
    return _import("bitpacking"), _import("bytepacking")


def load_gpu_variant():
    if not os.path.exists(_so("gpu_bitpacking")):
        build()
    return _import("gpu_bitpacking")


if __name__ == "__main__":
    ok = build(verbose="-v" in sys.argv)
    print("built" if ok else "reference absent: nothing built", OUT)
