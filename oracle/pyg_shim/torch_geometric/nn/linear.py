"""torch_geometric.nn.Linear (PyG 2.0.4) restated: `weight` [out, in], `bias` [out]."""
import math

import torch
from torch import nn
import torch.nn.functional as F


def _uniform(bound, t):
    with torch.no_grad():
        t.uniform_(-bound, bound)


class Linear(nn.Module):
    def __init__(self, in_channels, out_channels, bias=True, weight_initializer=None,
                 bias_initializer=None):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight_initializer = weight_initializer
        self.bias_initializer = bias_initializer
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.weight_initializer == "glorot":
            _uniform(math.sqrt(6.0 / (self.in_channels + self.out_channels)), self.weight)
        else:  # PyG 2.0.4 default: kaiming_uniform(fan=in, a=sqrt(5)) -> bound 1/sqrt(in)
            _uniform(1.0 / math.sqrt(self.in_channels), self.weight)
        if self.bias is not None:
            if self.bias_initializer == "zeros":
                with torch.no_grad():
                    self.bias.zero_()
            else:
                _uniform(1.0 / math.sqrt(self.in_channels), self.bias)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def __repr__(self):
        return f"Linear({self.in_channels}, {self.out_channels}, bias={self.bias is not None})"
