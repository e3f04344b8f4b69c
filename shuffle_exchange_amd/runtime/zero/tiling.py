"""``TiledLinear``: a Linear split into in_splits x out_splits tiles, each its own module.

Parity: reference runtime/zero/tiling.py:32 ``TiledLinear`` (and :259 ``TiledLinearReturnBias``).
Each tile is an element of a ``ModuleList``, so under ZeRO-3 (runtime/zero/stage3.py
``discover_units``) every tile is its own fetch unit: only one tile's weights are gathered at a time,
which bounds the memory of huge projections (e.g. a 128k-vocabulary LM head). On MI355X prefer
few, large tiles -- each tile is one hipBLASLt GEMM and should stay >= a few thousand columns.
"""
import torch
import torch.nn as nn


def _split(n, k):
    base, rem = divmod(n, k)
    return [base + (1 if i < rem else 0) for i in range(k)]


class TiledLinear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, in_splits=1, out_splits=1,
                 input_is_already_split=False, combine_out_splits=True, linear_cls=nn.Linear, init_linear=None,
                 **kwargs):
        super().__init__()
        assert 1 <= in_splits <= in_features and 1 <= out_splits <= out_features
        self.in_features, self.out_features = in_features, out_features
        self.in_splits, self.out_splits = in_splits, out_splits
        self.input_is_already_split, self.combine_out_splits = input_is_already_split, combine_out_splits
        self.in_parts, self.out_parts = _split(in_features, in_splits), _split(out_features, out_splits)
        self.use_bias = bias
        # tile (o, i) = linears[o * in_splits + i]; only the in_splits-1'th column of tiles has a bias
        tiles = []
        for o in range(out_splits):
            for i in range(in_splits):
                tiles.append(linear_cls(self.in_parts[i], self.out_parts[o], bias=bias and i == 0, **kwargs))
        self.linears = nn.ModuleList(tiles)
        if init_linear is not None:
            self.copy_params_from(init_linear)

    def tile(self, o, i):
        return self.linears[o * self.in_splits + i]

    def forward(self, x):
        xs = x if self.input_is_already_split else list(torch.split(x, self.in_parts, dim=-1))
        assert len(xs) == self.in_splits
        outs = []
        for o in range(self.out_splits):
            acc = None
            for i in range(self.in_splits):
                y = self.tile(o, i)(xs[i])
                acc = y if acc is None else acc + y
            outs.append(acc)
        return torch.cat(outs, dim=-1) if self.combine_out_splits else outs

    @torch.no_grad()
    def copy_params_from(self, other):
        """Copy the weights of a regular Linear into the tiles (reference tiling.py copy_params_from)."""
        assert other.weight.shape == (self.out_features, self.in_features)
        r0 = 0
        for o in range(self.out_splits):
            c0 = 0
            for i in range(self.in_splits):
                t = self.tile(o, i)
                t.weight.copy_(other.weight[r0:r0 + self.out_parts[o], c0:c0 + self.in_parts[i]])
                if t.bias is not None and other.bias is not None:
                    t.bias.copy_(other.bias[r0:r0 + self.out_parts[o]])
                c0 += self.in_parts[i]
            r0 += self.out_parts[o]


class TiledLinearReturnBias(TiledLinear):
    """Megatron-style: returns (output without bias, bias) (reference tiling.py:259)."""

    def forward(self, x):
        xs = x if self.input_is_already_split else list(torch.split(x, self.in_parts, dim=-1))
        outs, biases = [], []
        for o in range(self.out_splits):
            acc = None
            for i in range(self.in_splits):
                t = self.tile(o, i)
                y = torch.nn.functional.linear(xs[i], t.weight)
                acc = y if acc is None else acc + y
            outs.append(acc)
            b = self.tile(o, 0).bias
            biases.append(b)
        out = torch.cat(outs, dim=-1) if self.combine_out_splits else outs
        bias = (torch.cat(biases) if self.use_bias else None) if self.combine_out_splits else biases
        return out, bias
