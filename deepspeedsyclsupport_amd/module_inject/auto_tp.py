"""Automatic tensor parallelism for arbitrary HF models (reference `module_inject/auto_tp.py:186-500`,
`fusedqkv_utils.py`, `tp_shard.py`).

Walks the model, classifies each Linear / HF Conv1D inside a repeated block as
  * row-parallel ("all-reduce") if its name marks an output projection (o_proj, out_proj, down_proj, dense_4h_to_h,
    c_proj, fc2, fc_out, w2, wo, attention `dense`) -> `LinearAllreduce` with a column slice of W,
  * column-parallel otherwise -> `LinearLayer` with a row slice (fused QKV weights are sliced per q/k/v part or per
    head for interleaved layouts, so every rank keeps whole heads),
and divides the head-count attributes of attention modules so HF reshapes see the local head count.
Embeddings and the LM head stay replicated (vocab GEMM is cheap relative to 288 GB HBM).
"""
import re

import torch
import torch.nn as nn

from .layers import LinearAllreduce, LinearLayer

ROW_PARALLEL = ("o_proj", "out_proj", "down_proj", "dense_4h_to_h", "c_proj", "fc2", "fc_out", "w2", "wo",
                "proj_out")
ATTN_DENSE = re.compile(r"(attention|attn|self_attention)\.dense$")
FUSED_BLOCKS = ("c_attn", "qkv_proj", "Wqkv", "qkv")          # [q | k | v] stacked along the output dim
FUSED_INTERLEAVED = ("query_key_value", )                   # [heads, 3, D] interleaved (BLOOM / GPT-NeoX)
FUSED_GATE_UP = ("gate_up_proj", )
HEAD_ATTRS = ("num_heads", "num_attention_heads", "num_key_value_heads", "num_kv_heads", "n_head", "n_heads")
WIDTH_ATTRS = ("split_size", "all_head_size", "embed_dim", "hidden_size_per_partition", "inner_dim")


def _is_conv1d(m):
    return type(m).__name__ == "Conv1D" and hasattr(m, "nf")


def _linear_weight(m):
    """Return W as [out, in] regardless of Linear vs Conv1D."""
    return m.weight.data.t() if _is_conv1d(m) else m.weight.data


def _slice_rows(w, r, tp):
    n = w.shape[0] // tp
    return w[r * n:(r + 1) * n].contiguous()


class AutoTP:

    def __init__(self, model, mp_group, tp_size, tp_rank, kv_heads=None, injection_policy=None):
        """`injection_policy`: {block class: name or tuple of names of the linears whose output is all-reduced}
        (reference `inference/engine.py:135-154`, `module_inject/replace_module.py:266-300`): inside every instance
        of a listed class the named linears are split along their input features and all-reduced, every other
        linear of the block along its output features; nothing outside those blocks is touched."""
        self.policy = self._normalise_policy(injection_policy)
        self.model = model
        self.mp_group = mp_group
        self.tp = tp_size
        self.rank = tp_rank
        cfg = getattr(model, "config", None)
        self.num_heads = getattr(cfg, "num_attention_heads", None) or getattr(cfg, "n_head", None)
        self.kv_heads = kv_heads or getattr(cfg, "num_key_value_heads", None) or self.num_heads
        self.replaced = []

    # ------------------------------------------------------------------------------------------ policy
    @staticmethod
    def is_row_parallel(name):
        leaf = name.split(".")[-1]
        return leaf in ROW_PARALLEL or bool(ATTN_DENSE.search(name)) or name.endswith("output.dense")

    @staticmethod
    def in_block(name):
        return bool(re.search(r"\.(\d+)\.", "." + name + "."))

    # ------------------------------------------------------------------------------------------ slicing
    def _column(self, name, m):
        w = _linear_weight(m)
        b = m.bias.data if m.bias is not None else None
        leaf = name.split(".")[-1]
        r, tp = self.rank, self.tp
        if leaf in FUSED_BLOCKS and self.num_heads:
            D = w.shape[1] // self.num_heads
            sizes = [self.num_heads * D, self.kv_heads * D, self.kv_heads * D]
            if sum(sizes) != w.shape[0]:
                sizes = [w.shape[0] // 3] * 3
            parts = w.split(sizes, 0)
            w = torch.cat([_slice_rows(p, r, tp) for p in parts], 0)
            if b is not None:
                b = torch.cat([_slice_rows(p, r, tp) for p in b.split(sizes, 0)], 0)
        elif leaf in FUSED_GATE_UP:
            parts = w.chunk(2, 0)
            w = torch.cat([_slice_rows(p, r, tp) for p in parts], 0)
            if b is not None:
                b = torch.cat([_slice_rows(p, r, tp) for p in b.chunk(2, 0)], 0)
        else:  # plain or head-interleaved fused qkv: contiguous row slice keeps whole heads
            w = _slice_rows(w, r, tp)
            if b is not None:
                b = _slice_rows(b, r, tp)
        return LinearLayer(weight=nn.Parameter(w.contiguous(), requires_grad=False),
                           bias=None if b is None else nn.Parameter(b.contiguous(), requires_grad=False))

    def _row(self, name, m):
        w = _linear_weight(m)
        n = w.shape[1] // self.tp
        w = w[:, self.rank * n:(self.rank + 1) * n].contiguous()
        b = m.bias.data if m.bias is not None else None
        return LinearAllreduce(nn.Parameter(w, requires_grad=False),
                               None if b is None else nn.Parameter(b.clone(), requires_grad=False), self.mp_group)

    # ------------------------------------------------------------------------------------------ user policy
    @staticmethod
    def _normalise_policy(policy):
        if not policy:
            return None
        out = {}
        for cls, names in policy.items():
            if not (isinstance(cls, type) and issubclass(cls, nn.Module)):
                raise TypeError(f"{cls} is not a subclass of torch.nn.Module")
            out[cls] = (names, ) if isinstance(names, str) else tuple(names)
        return out

    @staticmethod
    def _ends_with(name, suffix):
        return ("." + name).endswith("." + suffix.lstrip("."))

    def _policy_targets(self):
        """(qualified name, module, is_row_parallel) of every linear inside a block the user policy lists."""
        all_names = [n for n, _ in self.model.named_modules()]
        for names in self.policy.values():
            for suffix in names:
                if not any(self._ends_with(n, suffix) for n in all_names):
                    raise ValueError(f"Injection policy layer '{suffix}' not valid.")
        seen, out = set(), []
        for bname, blk in self.model.named_modules():
            rows = next((v for k, v in self.policy.items() if isinstance(blk, k)), None)
            if rows is None:
                continue
            for rel, m in blk.named_modules():
                if not rel or not (isinstance(m, nn.Linear) or _is_conv1d(m)):
                    continue
                full = f"{bname}.{rel}" if bname else rel
                if full in seen:
                    continue
                seen.add(full)
                out.append((full, m, any(self._ends_with(rel, s) for s in rows)))
        return out

    @staticmethod
    def tp_parser(model):
        """[(block class, tuple of all-reduce linear names)] derived from the model's structure (reference
        `module_inject/auto_tp.py:271-311`): the repeated blocks are the children of ModuleLists; inside a block a
        linear is all-reduced when its name is a known output projection, when it is the last linear before a
        normalisation layer, or when it is the last linear of the block."""
        found = {}
        for _, lst in model.named_modules():
            if not isinstance(lst, nn.ModuleList) or len(lst) == 0:
                continue
            blk = lst[0]
            if sum(1 for _ in blk.modules()) < 3 or type(blk) in found:
                continue
            rows, last_linear = [], None
            for rel, m in blk.named_modules():
                if not rel:
                    continue
                if isinstance(m, nn.Linear) or _is_conv1d(m):
                    last_linear = rel
                    if AutoTP.is_row_parallel(rel):
                        rows.append(rel)
                elif "norm" in type(m).__name__.lower() or rel.split(".")[-1] in ("ln", "LayerNorm", "layer_norm"):
                    if last_linear is not None and last_linear not in rows:
                        rows.append(last_linear)
                    last_linear = None
            if last_linear is not None and last_linear not in rows:  # the block's output projection
                rows.append(last_linear)
            if rows:
                found[type(blk)] = tuple(dict.fromkeys(rows))
        if not found:
            raise ValueError("Not able to determine model policy automatically. Please provide policy.")
        return list(found.items())

    # ------------------------------------------------------------------------------------------ apply
    def apply(self):
        if self.tp <= 1:
            return self.model
        if self.policy is not None:
            targets = self._policy_targets()
        else:
            targets = []
            for name, m in self.model.named_modules():
                if (isinstance(m, nn.Linear) or _is_conv1d(m)) and self.in_block(name):
                    targets.append((name, m, self.is_row_parallel(name)))
        for name, m, row in targets:
            new = self._row(name, m) if row else self._column(name, m)
            parent_name, _, leaf = name.rpartition(".")
            parent = self.model.get_submodule(parent_name) if parent_name else self.model
            setattr(parent, leaf, new)
            self.replaced.append((name, type(new).__name__))
        self._fix_attrs()
        return self.model

    def _fix_attrs(self):
        in_policy = set()
        if self.policy is not None:  # the listed blocks (and what they contain) hold the head counts
            for _, blk in self.model.named_modules():
                if isinstance(blk, tuple(self.policy)):
                    in_policy.update(id(m) for m in blk.modules())
        for name, m in self.model.named_modules():
            if id(m) not in in_policy and not re.search(r"attn|attention", name.split(".")[-1] if name else "", re.I):
                continue
            for a in HEAD_ATTRS:
                v = getattr(m, a, None)
                if isinstance(v, int) and v >= self.tp and v % self.tp == 0:
                    setattr(m, a, v // self.tp)
            for a in WIDTH_ATTRS:
                v = getattr(m, a, None)
                if isinstance(v, int) and v % self.tp == 0:
                    setattr(m, a, v // self.tp)


def __getattr__(name):
    # `ReplaceWithTensorSlicing` is defined next to the whole-model replacement (replace_module.py imports this file)
    if name == "ReplaceWithTensorSlicing":
        from .replace_module import ReplaceWithTensorSlicing
        return ReplaceWithTensorSlicing
    raise AttributeError(name)


class Loading:
    """Which layer types are filled from a checkpoint's state dict while sharding a meta-device model (reference
    `auto_tp.py:124-183`)."""

    @staticmethod
    def is_load_module(module):
        names = ("LayerNorm", "Linear", "Embedding", "RMSNorm", "LPLayerNorm", "SharedEmbedding", "OPTLearnedPositionalEmbedding")
        return isinstance(module, (nn.Linear, nn.Embedding, nn.LayerNorm)) or \
            any(n.lower() in type(module).__name__.lower() for n in names)

    @staticmethod
    def load_buffer(module, state_dict, prefix):
        for name, buf in module.named_buffers(recurse=False):
            key = prefix + name
            if key in state_dict:
                src = state_dict[key]
                module._buffers[name] = src.to(buf.device if buf.device.type != "meta" else src.device)

    @staticmethod
    def load(module, state_dict, prefix, mp_group=None):
        """Fill `module`'s own parameters from `state_dict[prefix + name]`, materialising meta parameters."""
        for name, p in list(module.named_parameters(recurse=False)):
            key = prefix + name
            if key not in state_dict:
                continue
            src = state_dict[key]
            if p.device.type == "meta" or p.shape != src.shape:
                setattr(module, name, nn.Parameter(src.detach().clone(), requires_grad=p.requires_grad))
            else:
                with torch.no_grad():
                    p.copy_(src)
        Loading.load_buffer(module, state_dict, prefix)

