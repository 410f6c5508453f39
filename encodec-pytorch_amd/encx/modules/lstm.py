"""SLSTM (modules/lstm.py of the reference).

Phase-1 choice: the 2-layer LSTM(512) over 75 frames stays on the vendor RNN
(MIOpen through torch.nn.LSTM); it is a 20 GFLOP/step sequential recurrence and is the next
kernel to replace with a persistent-CU LSTM.
"""
from torch import nn


class SLSTM(nn.Module):
    """modules/lstm.py:12-28: permute to [T,B,C], LSTM, skip add, permute back."""

    def __init__(self, dimension: int, num_layers: int = 2, skip: bool = True):
        super().__init__()
        self.skip = skip
        self.lstm = nn.LSTM(dimension, dimension, num_layers)

    def forward(self, x):
        x = x.permute(2, 0, 1)
        y, _ = self.lstm(x)
        if self.skip:
            y = y + x
        return y.permute(1, 2, 0)
