"""Mirror of the reference's `modules` package (modules/__init__.py:10-22)."""
from .conv import (NormConv1d, NormConv2d, NormConvTranspose1d, SConv1d, SConvTranspose1d,  # noqa: F401
                   get_extra_padding_for_conv1d, CONV_NORMALIZATIONS)
from .lstm import SLSTM  # noqa: F401
from .seanet import SEANetEncoder, SEANetDecoder, SEANetResnetBlock  # noqa: F401
