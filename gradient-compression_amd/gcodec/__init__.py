"""gcodec — MI355X-native (gfx950) QSGD-MaxNorm gradient codec.

Hand-written HIP kernels (gradient-compression_amd/csrc) behind a C ABI
(include/gcodec.h), with drop-in Python classes named after the reference's
compressors.py / reducer.py / extensions.
"""
from . import codec  # noqa: F401
from ._lib import GCodecError  # noqa: F401
from .compressors import (  # noqa: F401
    GlobalRandKMaxNormCompressor,
    GlobalRandKMaxNormTwoScaleCompressor,
    QSGDBPCompressor,
    QSGDMaxNormCompressor,
    QSGDMaxNormMultiScaleCompressor,
    QSGDMaxNormTwoScaleCompressor,
)
from .reducer import (  # noqa: F401
    GlobalRandKMaxNormReducer,
    GlobalRandKMaxNormTwoScaleReducer,
    QSGDMaxNormMultiScaleReducer,
    QSGDMaxNormReducer,
    QSGDMaxNormTwoScaleReducer,
    Reducer,
    TensorBuffer,
    set_seed,
)
from .ddp_hook import QSGDHookState, qsgd_hook  # noqa: F401
from .pipeline import ChunkedQSGDAllReduce  # noqa: F401
from .rng import Generator, default_generator, manual_seed, set_mode  # noqa: F401
from .topology import NodeTopology  # noqa: F401

set_rng_mode = set_mode


def version() -> str:
    from ._lib import load

    return load().gc_version().decode()
