"""jwave_amd — MI355X (gfx950) engine for JWave's FWT / WPT / MODWT hot path.

Compute runs only in libjwave_hip.so (hand-written HIP kernels); this package
is the host mirror of the reference operator API over its C ABI
(include/jwave_hip.h).  See DESIGN.md.
"""
from .exceptions import JWaveError, JWaveException, JWaveFailure  # noqa: F401
from .wavelets import Wavelet, WaveletBuilder, by_class  # noqa: F401
from .transforms import (  # noqa: F401
    AncientEgyptianDecomposition, BasicTransform, CompressorMagnitude, Context, FastWaveletTransform,
    InPlaceFastWaveletTransform, MODWTTransform, MultiContext, ParallelTransform,
    ParallelWaveletPacketTransform,
    PooledWaveletPacketTransform, Transform, WaveletPacketTransform, WaveletTransform,
    batch_split, compress_magnitude, decompose_number, default_context, fwt_denoise, fwt_forward, fwt_reverse, modwt_filters, modwt_forward, modwt_inverse,
    transform_2d, transform_3d, transform_axis, wpt_forward, wpt_reverse)

__version__ = "0.1.0"
