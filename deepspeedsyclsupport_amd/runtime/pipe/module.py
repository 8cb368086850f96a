"""PipelineModule / LayerSpec / TiedLayerSpec (reference `runtime/pipe/module.py:30-636`).

The model is described as a flat list of layers (or LayerSpecs, built lazily so each stage only materialises its own
layers). Layers are partitioned over the pipeline stages by `partition_method`:
  "parameters" (balance trainable parameter counts), "uniform" (balance layer counts),
  "type:<regex>" (balance layers whose class name matches), or an explicit list of boundaries.
Tied layers (e.g. input embedding and LM head) are built on every stage that uses them; their gradients are summed
over the tie group and their weights broadcast from the first owner at init.
"""
import re
from functools import partial

import torch
import torch.nn as nn

from ... import comm as dist
from ...utils.logging import logger
from .topology import PipeDataParallelTopology, PipelineParallelGrid


class PipelineError(Exception):
    pass


class LayerSpec:

    def __init__(self, typename, *module_args, **module_kwargs):
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs
        if not issubclass(typename, nn.Module):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types.")
        self.global_rank = dist.get_rank() if dist.is_initialized() else -1

    def __repr__(self):
        return f"LayerSpec({self.typename.__name__})"

    def build(self, log=False):
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):

    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr="weight", **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = tied_weight_attr


def partition_uniform(num_items, num_parts):
    parts = [0] * (num_parts + 1)
    if num_items <= num_parts:
        for p in range(num_parts + 1):
            parts[p] = min(p, num_items)
        return parts
    chunk = num_items / num_parts
    for p in range(num_parts):
        parts[p] = int(round(chunk * p))
    parts[num_parts] = num_items
    return parts


def partition_balanced(weights, num_parts):
    """Contiguous partition minimising the max part weight (binary search over the bottleneck)."""
    n = len(weights)
    if num_parts >= n:
        return [min(i, n) for i in range(num_parts + 1)]
    prefix = [0]
    for w in weights:
        prefix.append(prefix[-1] + w)

    def parts_for(limit):
        parts = [0]
        start = 0
        for _ in range(num_parts):
            end = start
            while end < n and prefix[end + 1] - prefix[start] <= limit:
                end += 1
            if end == start and start < n:
                return None
            parts.append(end)
            start = end
        return parts if parts[-1] == n else None

    lo, hi = max(weights), prefix[-1]
    best = None
    while lo <= hi:
        mid = (lo + hi) // 2
        p = parts_for(mid)
        if p is not None:
            best, hi = p, mid - 1
        else:
            lo = mid + 1
    return best


class PipelineModule(nn.Module):

    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seed_layers=False, seed_fn=None,
                 base_seed=1234, partition_method="parameters", activation_checkpoint_interval=0,
                 activation_checkpoint_func=None, checkpointable_layers=None):
        super().__init__()
        if num_stages is None and topology is None:
            raise RuntimeError("must provide num_stages or topology")
        self.micro_offset = 0
        self.loss_fn = loss_fn
        self.checkpointable_layers = checkpointable_layers
        self.seed_layers = seed_layers
        self.seed_fn = seed_fn
        self.base_seed = base_seed
        self.world_group = dist.new_group(ranks=range(dist.get_world_size()))
        self.global_rank = dist.get_rank(group=self.world_group)
        self.world_size = dist.get_world_size(group=self.world_group)
        self.local_rank = int(__import__("os").environ.get("LOCAL_RANK", "0"))
        if topology:
            self._topo = topology
            self.num_stages = self._topo.get_dim("pipe")
        else:
            self.num_stages = num_stages
            self._topo = PipeDataParallelTopology(num_pp=num_stages, num_dp=self.world_size // num_stages)
        self._grid = PipelineParallelGrid(process_group=self.world_group, topology=self._topo)
        self.stage_id = self._topo.get_coord(self.global_rank).pipe
        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self._local_start = 0
        self._local_stop = None
        self._partition_layers(method=partition_method)
        self.forward_funcs = []
        self.fwd_map = {}
        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs = {}
        self._build()
        self.tied_comms = self._index_tied_modules()
        self._synchronize_tied_weights()
        self.activation_checkpoint_interval = activation_checkpoint_interval
        if activation_checkpoint_func is None:
            from ..activation_checkpointing import checkpointing
            activation_checkpoint_func = checkpointing.checkpoint
        self.activation_checkpoint_func = activation_checkpoint_func

    # ------------------------------------------------------------------------------------------ build
    def _build(self):
        specs = self._layer_specs
        for local_idx, layer in enumerate(specs[self._local_start:self._local_stop]):
            layer_idx = local_idx + self._local_start
            if self.seed_layers:
                (self.seed_fn or torch.manual_seed)(self.base_seed + layer_idx)
            if isinstance(layer, nn.Module):
                name = str(layer_idx)
                self.forward_funcs.append(layer)
                self.fwd_map[name] = len(self.forward_funcs) - 1
                self.add_module(name, layer)
            elif isinstance(layer, TiedLayerSpec):
                if layer.key not in self.tied_modules:
                    self.tied_modules[layer.key] = layer.build()
                    self.tied_weight_attrs[layer.key] = layer.tied_weight_attr
                if layer.forward_fn is None:
                    self.forward_funcs.append(self.tied_modules[layer.key])
                else:
                    self.forward_funcs.append(partial(layer.forward_fn, self.tied_modules[layer.key]))
            elif isinstance(layer, LayerSpec):
                module = layer.build()
                name = str(layer_idx)
                self.forward_funcs.append(module)
                self.fwd_map[name] = len(self.forward_funcs) - 1
                self.add_module(name, module)
            else:
                self.forward_funcs.append(layer)  # plain callable (e.g. lambda reshape)

    def _count_layer_params(self):
        counts = []
        for layer in self._layer_specs:
            if isinstance(layer, LayerSpec):
                m = layer.build()
                counts.append(sum(p.numel() for p in m.parameters() if p.requires_grad))
            elif isinstance(layer, nn.Module):
                counts.append(sum(p.numel() for p in layer.parameters() if p.requires_grad))
            else:
                counts.append(0)
        return counts

    def _find_layer_type(self, layername):
        idxs = []
        typeregex = re.compile(layername, re.IGNORECASE)
        for idx, layer in enumerate(self._layer_specs):
            name = None
            if isinstance(layer, LayerSpec):
                name = layer.typename.__name__
            elif isinstance(layer, nn.Module):
                name = layer.__class__.__name__
            else:
                try:
                    name = layer.__name__
                except AttributeError:
                    continue
            if typeregex.search(name):
                idxs.append(idx)
        if len(idxs) == 0:
            raise RuntimeError(f"Partitioning '{layername}' found no valid layers to partition.")
        return idxs

    def _partition_layers(self, method="uniform"):
        num_stages = self._topo.get_dim("pipe")
        stage_id = self._topo.get_coord(self.global_rank).pipe
        if isinstance(method, (list, tuple)):
            self.parts = list(method)
        else:
            method = method.lower()
            if method == "uniform":
                self.parts = partition_uniform(num_items=self._num_layers, num_parts=num_stages)
            elif method == "parameters":
                counts = self._count_layer_params()
                self.parts = partition_balanced(weights=[max(c, 1) for c in counts], num_parts=num_stages)
            elif method.startswith("type:"):
                layertype = method.split(":")[1]
                binary = [0] * len(self._layer_specs)
                for idx in self._find_layer_type(layertype):
                    binary[idx] = 1
                self.parts = partition_balanced(weights=[b * 1000 + 1 for b in binary], num_parts=num_stages)
            elif method == "profile":
                raise NotImplementedError(f"Partitioning method {method} not implemented.")
            else:
                raise NotImplementedError(f"Partitioning method {method} not implemented.")
        self._set_bounds(start=self.parts[stage_id], stop=self.parts[stage_id + 1])

    def _set_bounds(self, start=None, stop=None):
        self._local_start = start
        self._local_stop = stop

    # ------------------------------------------------------------------------------------------ tied weights
    def _index_tied_modules(self):
        tied_comms = {}
        if self._topo.get_dim("pipe") == 1:
            return tied_comms
        specs = self._layer_specs
        tie_keys = set(s.key for s in specs if isinstance(s, TiedLayerSpec))
        for key in sorted(tie_keys):
            tied_layers = [i for i, s in enumerate(specs) if isinstance(s, TiedLayerSpec) and s.key == key]
            tied_stages = sorted(set(self.stage_owner(i) for i in tied_layers))
            for dp in range(self._grid.data_parallel_size):
                for mp in range(self._grid.get_slice_parallel_world_size()):
                    tied_ranks = []
                    for s in tied_stages:
                        if self._grid.get_slice_parallel_world_size() > 1:
                            tied_ranks.append(self._grid.stage_to_global(stage_id=s, data=dp, model=mp))
                        else:
                            tied_ranks.append(self._grid.stage_to_global(stage_id=s, data=dp))
                    group = dist.new_group(ranks=tied_ranks)
                    if self.global_rank in tied_ranks:
                        assert key in self.tied_modules
                        tied_comms[key] = {
                            "ranks": tied_ranks,
                            "group": group,
                            "weight_attr": self.tied_weight_attrs[key],
                            "module": self.tied_modules[key],
                        }
        return tied_comms

    def _synchronize_tied_weights(self):
        for key, comm in self.tied_comms.items():
            w = getattr(comm["module"], comm["weight_attr"])
            dist.broadcast(w.data, src=min(comm["ranks"]), group=comm["group"])

    def allreduce_tied_weight_gradients(self):
        for key, comm in self.tied_comms.items():
            w = getattr(comm["module"], comm["weight_attr"])
            if w.grad is not None:
                dist.all_reduce(w.grad, group=comm["group"])

    def get_tied_weights_and_groups(self):
        return [(getattr(c["module"], c["weight_attr"]), c["group"]) for c in self.tied_comms.values()]

    # ------------------------------------------------------------------------------------------ forward
    def forward(self, forward_input):
        self.micro_offset += 1

        def exec_range_func(start, end):
            local_micro_offset = self.micro_offset + 1

            def exec_func(*inputs):
                if len(inputs) == 1:
                    inputs = inputs[0]
                for idx, layer in enumerate(self.forward_funcs[start:end]):
                    self.curr_layer = idx + self._local_start
                    if self.seed_layers:
                        new_seed = (self.base_seed * local_micro_offset) + self.curr_layer
                        (self.seed_fn or torch.manual_seed)(new_seed)
                    inputs = layer(inputs)
                return inputs

            return exec_func

        if self.activation_checkpoint_interval == 0 or not self.training:
            return exec_range_func(0, len(self.forward_funcs))(forward_input)
        num_layers = len(self.forward_funcs)
        x = forward_input
        for start_idx in range(0, num_layers, self.activation_checkpoint_interval):
            end_idx = min(start_idx + self.activation_checkpoint_interval, num_layers)
            funcs = self.forward_funcs[start_idx:end_idx]
            if not isinstance(x, tuple):
                x = (x, )
            if self._is_checkpointable(funcs):
                x = self.activation_checkpoint_func(exec_range_func(start_idx, end_idx), *x)
            else:
                x = exec_range_func(start_idx, end_idx)(*x)
        return x

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(f.__class__.__name__ in self.checkpointable_layers for f in funcs)
        params = [f.parameters() for f in funcs if isinstance(f, nn.Module)]
        return any(len(list(p)) > 0 for p in params)

    # ------------------------------------------------------------------------------------------ misc
    def stage_owner(self, layer_idx):
        assert 0 <= layer_idx < self._num_layers
        for stage in range(self._topo.get_dim("pipe")):
            if self.parts[stage] <= layer_idx < self.parts[stage + 1]:
                return stage
        raise RuntimeError(f"Layer {layer_idx} not owned? parts={self.parts}")

    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def num_pipeline_stages(self):
        return self._topo.get_dim("pipe")

    def ckpt_prefix(self, checkpoints_path, tag):
        import os
        return os.path.join(checkpoints_path, str(tag))

    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        import os
        idx = local_layer_idx + self._local_start
        layer_ckpt_path = os.path.join(ckpt_dir, f"layer_{idx:02d}")
        rank_repr = self._grid._topo.get_rank_repr(rank=self.global_rank)
        if rank_repr != "":
            layer_ckpt_path += f"-{rank_repr}"
        layer_ckpt_path += "-model_states.pt"
        return layer_ckpt_path
