"""Mirror of the reference's `quantization` package (quantization/__init__.py)."""
from .vq import QuantizedResult, ResidualVectorQuantizer  # noqa: F401
