"""TiledLinear (reference `runtime/zero/tiling.py:32-296`): a Linear split into in_splits x out_splits tiles, each its
own module, so ZeRO-3 gathers (and frees) one tile's weights at a time instead of the whole matrix."""
import torch
import torch.nn as nn


def split_tensor_along_last_dim(x, partitions):
    sizes = partitions if isinstance(partitions, (list, tuple)) else _split_sizes(x.shape[-1], partitions)
    return list(torch.split(x, sizes, dim=-1))


def _split_sizes(n, parts):
    base, rem = divmod(n, parts)
    return [base + (1 if i < rem else 0) for i in range(parts)]


class TiledLinear(nn.Module):

    def __init__(self, in_features, out_features, bias=True, in_splits=1, out_splits=1,
                 input_is_already_split=False, combine_out_splits=True, linear_cls=nn.Linear, init_linear=None,
                 **kwargs):
        super().__init__()
        if in_splits < 1 or in_splits > in_features or out_splits < 1 or out_splits > out_features:
            raise RuntimeError("in/out splits must be in [1, features]")
        self.in_features, self.out_features = in_features, out_features
        self.use_bias = bias
        self.in_splits, self.out_splits = in_splits, out_splits
        self.input_is_already_split = input_is_already_split
        self.combine_out_splits = combine_out_splits
        self.in_parts = _split_sizes(in_features, in_splits)
        self.out_parts = _split_sizes(out_features, out_splits)
        # bias lives only in the in-tile 0 of each out split (added once)
        self.linears = nn.ModuleList([
            nn.ModuleList([linear_cls(self.in_parts[i], self.out_parts[o], bias=bias and i == 0, **kwargs)
                           for i in range(in_splits)]) for o in range(out_splits)
        ])
        if init_linear is not None:
            self.copy_params_from(init_linear)

    def forward(self, input_):
        if self.in_splits > 1 and not self.input_is_already_split:
            inputs = split_tensor_along_last_dim(input_, self.in_parts)
        elif self.in_splits > 1:
            inputs = input_
            assert len(inputs) == self.in_splits
        else:
            inputs = [input_]
        outs = []
        for o in range(self.out_splits):
            acc = None
            for i in range(self.in_splits):
                y = self.linears[o][i](inputs[i])
                acc = y if acc is None else acc + y
            outs.append(acc)
        if self.combine_out_splits:
            return torch.cat(outs, dim=-1)
        return outs

    @torch.no_grad()
    def copy_params_from(self, other):
        """Copy weights (and bias) of a full nn.Linear into the tiles."""
        assert other.weight.shape == (self.out_features, self.in_features)
        ro = 0
        for o in range(self.out_splits):
            ri = 0
            for i in range(self.in_splits):
                t = self.linears[o][i]
                t.weight.copy_(other.weight[ro:ro + self.out_parts[o], ri:ri + self.in_parts[i]])
                if t.bias is not None and other.bias is not None:
                    t.bias.copy_(other.bias[ro:ro + self.out_parts[o]])
                ri += self.in_parts[i]
            ro += self.out_parts[o]


class TiledLinearReturnBias(TiledLinear):
    """Variant for layers that return (output, bias) (Megatron style)."""

    def forward(self, input_):
        out = super().forward(input_)
        return out, None
