"""encx -- MI355X-native (gfx950) EnCodec training hot path.

Host mirror of the reference's interfaces (EncodecModel, SEANet modules, RVQ, Audio2Mel,
losses, Balancer, schedulers, distrib) over libencx.so, the HIP kernels declared in
include/encx.h. Importing encx does not touch the GPU; the first op loads the library and
raises if it is missing (there is no CPU fallback).
"""
from ._lib import lib, LIB_PATH  # noqa: F401
from .model import EncodecModel  # noqa: F401
from .balancer import Balancer  # noqa: F401

__version__ = '0.1.0'
