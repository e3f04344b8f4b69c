"""ZeRO-3-safe linear (reference runtime/zero/linear.py:50 ``LinearFunctionForZeroStage3``, :121
``LinearModuleForZeroStage3``, ``zero3_linear_wrap``).

The reference needs its own autograd function so that ZeRO-3 can free the gathered weight after
the forward. Here ``ops.linear`` already does that job: its backward writes the weight gradient
straight into the unit's flat gradient staging buffer (TN-layout hipBLASLt GEMM when faster) and
stage 3 re-gathers or keeps the weight per its reuse policy, so the same function serves ZeRO-3 and
plain use."""
import torch

from ...ops.linear import _Linear, linear

LinearFunctionForZeroStage3 = _Linear


def zero3_linear_wrap(input, weight, bias=None):
    return linear(input, weight, bias)


class LinearModuleForZeroStage3(torch.nn.Linear):
    def forward(self, input):
        return linear(input, self.weight, self.bias)
