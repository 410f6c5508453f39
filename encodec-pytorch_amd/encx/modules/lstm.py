"""SLSTM (modules/lstm.py of the reference) on the encx LSTM kernels (csrc/lstm.hip).

The parameters stay in a torch.nn.LSTM container so the state-dict keys
(`lstm.weight_ih_l0`, `lstm.bias_hh_l1`, ...) and the default init match the reference;
its forward is never called: the sequence runs through encx.ops.LSTMFn.
"""
from torch import nn

from .. import ops


class SLSTM(nn.Module):
    """modules/lstm.py:12-28: permute to [T,B,C], LSTM, skip add, permute back."""

    def __init__(self, dimension: int, num_layers: int = 2, skip: bool = True):
        super().__init__()
        self.skip = skip
        self.lstm = nn.LSTM(dimension, dimension, num_layers)

    def _weights(self):
        w = []
        for l in range(self.lstm.num_layers):
            w += [getattr(self.lstm, f'{n}_l{l}')
                  for n in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh')]
        return w

    def forward(self, x):
        return ops.lstm(x, self._weights(), skip=self.skip)
