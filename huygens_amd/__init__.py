"""huygens_amd -- MI355X-native (gfx950 HIP) engine for the amcerbu/huygens bank hot path.

The product is libhuygens_hip.so (C ABI: include/huygens_hip.h) with the C++
drop-in headers in include/soundmath/.  This package is the Python mirror of
that ABI used by tests/ and bench.py.
"""
from ._lib import HZError, load, header_symbols, rt_info  # noqa: F401
from .filterbank import Filterbank, sample_many  # noqa: F401
from .oscbank import Oscbank  # noqa: F401
from .additive import Additive, Sinusoids  # noqa: F401
from .bowl import Bowl  # noqa: F401
from .delay import Delay, Delaybank  # noqa: F401
from .stft import Cosine, Fourier, StaticSTFT  # noqa: F401
from .granulator import GRAIN_REQ, Granulator  # noqa: F401
from .freezer import Freezer  # noqa: F401
from .heterodyne import Heterodyne, harmbank  # noqa: F401

__all__ = ["HZError", "load", "header_symbols", "Filterbank", "sample_many", "Oscbank", "Additive", "Sinusoids", "Bowl", "Delay", "Delaybank", "Fourier", "StaticSTFT", "Cosine", "Granulator", "GRAIN_REQ", "Freezer", "Heterodyne", "harmbank"]
