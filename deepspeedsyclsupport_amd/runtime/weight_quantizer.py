"""Int8 quantisation of Megatron-style checkpoint weights at load time (reference `runtime/weight_quantizer.py:10`
`WeightQuantization`): group-wise symmetric codes with one scale per group, an extra split of the MLP weights'
groups (`mlp_extra_grouping`, the 4h matrices are 4x taller/wider), and the per-layer scale table the kernel-injected
inference layers consume — rows [qkv, attn-out, h->4h, 4h->h], each padded to the widest.

Scales are returned as the dequantisation multiplier (`w ~= q * scale`), as in the reference (which stores
1 / quantisation-scale)."""
import torch

_QKV, _DENSE, _H4H, _4HH = "attention.query_key_value.weight", "attention.dense.weight", \
    "mlp.dense_h_to_4h.weight", "mlp.dense_4h_to_h.weight"
QUANTIZED_KEYS = (_QKV, _DENSE, _H4H, _4HH)


class WeightQuantization:

    def __init__(self, mlp_extra_grouping=True, mp_size=1):
        self.mlp_extra_grouping = mlp_extra_grouping
        self.mp_size = mp_size
        self.scales = {_QKV: [], _DENSE: [], _H4H: [], _4HH: []}

    # ------------------------------------------------------------------------------------------ primitives
    @staticmethod
    def quantize_data(data, quantize_bits, groups, key=None):
        """(int8 codes shaped like `data`, per-group quantisation scales [groups, 1])."""
        g = data.float().reshape(groups, -1)
        amax = g.abs().amax(dim=1, keepdim=True)
        qscale = float(1 << quantize_bits) / (2 * amax + 1e-5)
        lim = 1 << (quantize_bits - 1)
        q = torch.clamp(torch.round(g * qscale), -lim, lim - 1).to(torch.int8)
        return q.reshape(data.shape), qscale

    def is_mlp(self, data, merge_count=1):
        r, c = data.shape[0], data.shape[1]
        return self.mp_size * r * merge_count == 4 * c or self.mp_size * c * merge_count == 4 * r

    def is_qkv(self, data):
        r, c = data.shape[0], data.shape[1]
        return self.mp_size * r == 3 * c or self.mp_size * c == 3 * r

    def _slot(self, key):
        for k in (_4HH, _H4H, _QKV):
            if k in key:
                return k
        return _DENSE

    def Quantize(self, value_list, quantize_bits, groups, key, merge_dim=0):
        """Quantise every shard of one weight; record the concatenated dequant scales under the weight's role."""
        if self.mlp_extra_grouping and self.is_mlp(value_list[0], merge_count=len(value_list)):
            groups *= 2
        codes, scales = [], []
        for v in value_list:
            q, s = self.quantize_data(v, quantize_bits, groups, key)
            codes.append(q)
            scales.append(s)
        self.scales[self._slot(key)].append((1.0 / torch.cat(scales, dim=merge_dim)).reshape(1, -1))
        return codes

    # ------------------------------------------------------------------------------------------ scale tables
    @staticmethod
    def merge_layer_scales(layer_scales):
        width = max(s.shape[-1] for s in layer_scales)
        rows = [torch.nn.functional.pad(s, (0, width - s.shape[-1])) for s in layer_scales]
        return torch.cat(rows).unsqueeze(0)

    def _layers(self):
        return zip(self.scales[_QKV], self.scales[_DENSE], self.scales[_H4H], self.scales[_4HH])

    def merge_scales(self):
        """[layers, 4, width]: per layer (qkv, attn-out, h->4h, 4h->h)."""
        return torch.cat([self.merge_layer_scales(list(l)) for l in self._layers()])

    def merge_scales_split(self, split_count):
        """Per model-parallel slice: the same table cut into `split_count` column ranges, each row zero-padded to
        the widest (the MLP rows carry the doubled group count)."""
        out = [[] for _ in range(split_count)]
        for layer in self._layers():
            parts = [torch.chunk(t, split_count, dim=1) for t in layer]
            for s in range(split_count):
                out[s].append(self.merge_layer_scales([p[s] for p in parts]))
        return [torch.cat(rows) for rows in out]

    def sd_quantize_megatron(self, sd, quantize_bits, groups):
        for key in list(sd.keys()):
            if any(k in key for k in QUANTIZED_KEYS):
                sd[key] = self.Quantize([sd[key]], quantize_bits, groups, key=key)[0]
        return sd, self.merge_scales()

    def model_quantize(self, model, quantize_policy, quantize_bits, groups):
        """Quantise the four projection weights of every layer matched by `quantize_policy` ({layer class:
        callable(layer) -> (qkv_w, out_w, h4h_w, 4hh_w)}) in place; returns (model, [layers, 4, width] scales)."""
        tables = []
        for m in model.modules():
            getter = quantize_policy.get(type(m)) if quantize_policy else None
            if getter is None:
                continue
            row = []
            for w in getter(m):
                g = groups * 2 if self.mlp_extra_grouping and self.is_mlp(w) else groups
                q, s = self.quantize_data(w.data, quantize_bits, g)
                w.data = q
                row.append((1.0 / s).reshape(1, -1))
            tables.append(self.merge_layer_scales(row))
        return model, (torch.cat(tables) if tables else None)
