"""neo (MI355X): the FFT + UPOLS hot path of neo-dsp on HIP/gfx950.

`import neo` mirrors the reference's Python package entry points that exist on
this path (extra/python/src/neo/__init__.py, neo/fft/__init__.py); the compute
is libneo_hip.so (include/neo_hip.h). Put `<repo>/neo-dsp_amd` on sys.path.
"""
from . import _native
from . import convolution
from . import fft
from .convolution import (UpolsConvolver, UpolsMultiConvolver, convolve, dense_convolve, direct_convolve, fft_convolve,
                          host_register, host_unregister, memory_info, memory_trim, normalize_impulse, overlap_add, overlap_save, OverlapStage, UpolsGroup,
                          num_partitions, split_upola_convolver, split_upols_convolver, uniform_partition,
                          upola_convolver, upola_convolver_v2, upols_convolver)

__version__ = "0.1.0"

__all__ = [
    "fft",
    "convolution",
    "UpolsConvolver",
    "UpolsMultiConvolver",
    "upols_convolver",
    "split_upols_convolver",
    "upola_convolver",
    "split_upola_convolver",
    "upola_convolver_v2",
    "uniform_partition",
    "normalize_impulse",
    "num_partitions",
    "overlap_save",
    "overlap_add",
    "OverlapStage",
    "UpolsGroup",
    "host_register",
    "host_unregister",
    "memory_info",
    "memory_trim",
    "dense_convolve",
    "convolve",
    "fft_convolve",
    "direct_convolve",
]
