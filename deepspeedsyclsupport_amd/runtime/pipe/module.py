"""PipelineModule / LayerSpec / TiedLayerSpec (API of the reference `runtime/pipe/module.py:30-636`).

The model is a flat sequence of entries — modules, LayerSpecs (built lazily, so a stage only materialises its own
layers), TiedLayerSpecs (one module shared by several positions, e.g. input embedding and LM head) or plain callables.
The sequence is cut into `num_stages` contiguous ranges by `partition_method`:
  "parameters"   — balance trainable parameter counts,
  "uniform"      — balance entry counts,
  "type:<regex>" — balance the entries whose class name matches,
  or an explicit list of stage boundaries.
Tied modules exist on every stage that uses them; their weights are broadcast from the lowest rank of the tie group at
construction and their gradients summed over it before the optimizer step.
"""
import os
import re
from functools import partial

import torch
import torch.nn as nn

from ... import comm as dist
from .topology import PipeDataParallelTopology, PipelineParallelGrid


class PipelineError(Exception):
    pass


class LayerSpec:
    """A deferred `typename(*args, **kwargs)`: only the owning stage pays for construction."""

    def __init__(self, typename, *module_args, **module_kwargs):
        if not (isinstance(typename, type) and issubclass(typename, nn.Module)):
            raise RuntimeError("LayerSpec only supports torch.nn.Module types.")
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs
        self.global_rank = dist.get_rank() if dist.is_initialized() else -1

    def __repr__(self):
        return f"LayerSpec({self.typename.__name__})"

    def build(self, log=False):
        return self.typename(*self.module_args, **self.module_kwargs)


class TiedLayerSpec(LayerSpec):
    """A LayerSpec whose module is shared by every entry with the same `key` (one instance per stage)."""

    def __init__(self, key, typename, *module_args, forward_fn=None, tied_weight_attr="weight", **module_kwargs):
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = tied_weight_attr


def partition_uniform(num_items, num_parts):
    """Boundaries [b0=0, ..., b_parts=num_items] with item counts differing by at most one."""
    if num_items <= num_parts:
        return [min(p, num_items) for p in range(num_parts + 1)]
    return [round(p * num_items / num_parts) for p in range(num_parts)] + [num_items]


def partition_balanced(weights, num_parts):
    """Contiguous partition minimising the heaviest part: binary search on that bound, greedy feasibility check."""
    n = len(weights)
    if num_parts >= n:
        return [min(i, n) for i in range(num_parts + 1)]
    prefix = [0]
    for w in weights:
        prefix.append(prefix[-1] + w)

    def cut(bound):
        bounds, start = [0], 0
        for _ in range(num_parts):
            end = start
            while end < n and prefix[end + 1] - prefix[start] <= bound:
                end += 1
            if end == start and start < n:
                return None
            bounds.append(end)
            start = end
        return bounds if bounds[-1] == n else None

    lo, hi, best = max(weights), prefix[-1], None
    while lo <= hi:
        mid = (lo + hi) // 2
        b = cut(mid)
        if b is None:
            lo = mid + 1
        else:
            best, hi = b, mid - 1
    return best


def _entry_name(entry):
    if isinstance(entry, LayerSpec):
        return entry.typename.__name__
    if isinstance(entry, nn.Module):
        return type(entry).__name__
    return getattr(entry, "__name__", None)


def _entry_params(entry):
    module = entry.build() if isinstance(entry, LayerSpec) else entry
    if not isinstance(module, nn.Module):
        return 0
    return sum(p.numel() for p in module.parameters() if p.requires_grad)


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
        self.seed_layers, self.seed_fn, self.base_seed = seed_layers, seed_fn, base_seed
        self.world_group = dist.new_group(ranks=range(dist.get_world_size()))
        self.global_rank = dist.get_rank(group=self.world_group)
        self.world_size = dist.get_world_size(group=self.world_group)
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self._topo = topology or PipeDataParallelTopology(num_pp=num_stages, num_dp=self.world_size // num_stages)
        self.num_stages = self._topo.get_dim("pipe")
        self._grid = PipelineParallelGrid(process_group=self.world_group, topology=self._topo)
        self.stage_id = self._topo.get_coord(self.global_rank).pipe
        self._layer_specs = list(layers)
        self._num_layers = len(self._layer_specs)
        self.parts = self._stage_boundaries(partition_method)
        self._local_start, self._local_stop = self.parts[self.stage_id], self.parts[self.stage_id + 1]
        self.forward_funcs, self.fwd_map = [], {}
        self.tied_modules, self.tied_weight_attrs = nn.ModuleDict(), {}
        for idx in range(self._local_start, self._local_stop):
            self._materialize(idx)
        self.tied_comms = self._index_tied_modules()
        self._synchronize_tied_weights()
        self.activation_checkpoint_interval = activation_checkpoint_interval
        if activation_checkpoint_func is None:
            from ..activation_checkpointing import checkpointing
            activation_checkpoint_func = checkpointing.checkpoint
        self.activation_checkpoint_func = activation_checkpoint_func
        # layer files written by every data-parallel replica (an even share each) instead of replica 0 alone; the
        # pipeline engine sets it from checkpoint.parallel_write.pipeline_stage
        self.checkpoint_parallel_write_pipeline = False

    # ------------------------------------------------------------------------------------------ partitioning
    def _stage_boundaries(self, method):
        if isinstance(method, (list, tuple)):
            bounds = [int(b) for b in method]
            if len(bounds) != self.num_stages + 1 or bounds[0] != 0 or bounds[-1] != self._num_layers:
                raise PipelineError(f"explicit partition {bounds} does not cover {self._num_layers} layers")
            return bounds
        method = method.lower()
        if method == "uniform":
            return partition_uniform(self._num_layers, self.num_stages)
        if method == "parameters":
            return partition_balanced([max(_entry_params(e), 1) for e in self._layer_specs], self.num_stages)
        if method.startswith("type:"):
            pattern = re.compile(method.split(":", 1)[1], re.IGNORECASE)
            hits = [bool(_entry_name(e) and pattern.search(_entry_name(e))) for e in self._layer_specs]
            if not any(hits):
                raise RuntimeError(f"Partitioning '{method}' found no valid layers to partition.")
            # matching layers dominate the balance; the +1 keeps the partition contiguous and total
            return partition_balanced([1000 * h + 1 for h in hits], self.num_stages)
        raise NotImplementedError(f"Partitioning method {method} not implemented.")

    def _set_bounds(self, start=None, stop=None):
        self._local_start, self._local_stop = start, stop

    def stage_owner(self, layer_idx):
        if not 0 <= layer_idx < self._num_layers:
            raise AssertionError(f"layer {layer_idx} out of range")
        for stage in range(self.num_stages):
            if self.parts[stage] <= layer_idx < self.parts[stage + 1]:
                return stage
        raise RuntimeError(f"Layer {layer_idx} not owned? parts={self.parts}")

    # ------------------------------------------------------------------------------------------ construction
    def _materialize(self, idx):
        entry = self._layer_specs[idx]
        if self.seed_layers:
            (self.seed_fn or torch.manual_seed)(self.base_seed + idx)
        if isinstance(entry, TiedLayerSpec):
            if entry.key not in self.tied_modules:
                self.tied_modules[entry.key] = entry.build()
                self.tied_weight_attrs[entry.key] = entry.tied_weight_attr
            shared = self.tied_modules[entry.key]
            self.forward_funcs.append(shared if entry.forward_fn is None else partial(entry.forward_fn, shared))
            return
        module = entry.build() if isinstance(entry, LayerSpec) else entry
        self.forward_funcs.append(module)
        if isinstance(module, nn.Module):
            self.fwd_map[str(idx)] = len(self.forward_funcs) - 1
            self.add_module(str(idx), module)

    # ------------------------------------------------------------------------------------------ tied weights
    def _index_tied_modules(self):
        """One group per (tie key, data replica, model slice) over the stages that hold the tied module."""
        comms = {}
        if self.num_stages == 1:
            return comms
        specs = self._layer_specs
        keys = sorted({s.key for s in specs if isinstance(s, TiedLayerSpec)})
        slices = self._grid.get_slice_parallel_world_size()
        for key in keys:
            stages = sorted({self.stage_owner(i) for i, s in enumerate(specs)
                             if isinstance(s, TiedLayerSpec) and s.key == key})
            for dp in range(self._grid.data_parallel_size):
                for mp in range(slices):
                    extra = {"data": dp}
                    if slices > 1:
                        extra["model"] = mp
                    ranks = [self._grid.stage_to_global(stage_id=s, **extra) for s in stages]
                    group = dist.new_group(ranks=ranks)
                    if self.global_rank in ranks:
                        comms[key] = {"ranks": ranks, "group": group, "weight_attr": self.tied_weight_attrs[key],
                                      "module": self.tied_modules[key]}
        return comms

    def _tied_weight(self, comm):
        return getattr(comm["module"], comm["weight_attr"])

    def _synchronize_tied_weights(self):
        for comm in self.tied_comms.values():
            dist.broadcast(self._tied_weight(comm).data, src=min(comm["ranks"]), group=comm["group"])

    def allreduce_tied_weight_gradients(self):
        for comm in self.tied_comms.values():
            w = self._tied_weight(comm)
            if w.grad is not None:
                dist.all_reduce(w.grad, group=comm["group"])

    def get_tied_weights_and_groups(self):
        return [(self._tied_weight(c), c["group"]) for c in self.tied_comms.values()]

    # ------------------------------------------------------------------------------------------ forward
    def _segment(self, start, end):
        """Callable running local entries [start, end); with seed_layers every layer reseeds from (micro-batch,
        layer index) so recomputation under activation checkpointing replays the same dropout masks."""
        micro = self.micro_offset + 1

        def run(*inputs):
            x = inputs[0] if len(inputs) == 1 else inputs
            for j, fn in enumerate(self.forward_funcs[start:end]):
                self.curr_layer = self._local_start + start + j
                if self.seed_layers:
                    (self.seed_fn or torch.manual_seed)(self.base_seed * micro + self.curr_layer)
                x = fn(x)
            return x

        return run

    def forward(self, forward_input):
        self.micro_offset += 1
        n = len(self.forward_funcs)
        interval = self.activation_checkpoint_interval
        if interval == 0 or not self.training:
            return self._segment(0, n)(forward_input)
        x = forward_input
        for lo in range(0, n, interval):
            hi = min(lo + interval, n)
            args = x if isinstance(x, tuple) else (x, )
            seg = self._segment(lo, hi)
            x = self.activation_checkpoint_func(seg, *args) if self._is_checkpointable(self.forward_funcs[lo:hi]) \
                else seg(*args)
        return x

    def _is_checkpointable(self, funcs):
        if self.checkpointable_layers is not None:
            return all(type(f).__name__ in self.checkpointable_layers for f in funcs)
        return any(isinstance(f, nn.Module) and any(True for _ in f.parameters()) for f in funcs)

    # ------------------------------------------------------------------------------------------ misc
    def topology(self):
        return self._topo

    def mpu(self):
        return self._grid

    def num_pipeline_stages(self):
        return self.num_stages

    def partitions(self):
        """Stage boundaries over the layer list: stage s runs layers [parts[s], parts[s + 1])."""
        return self.parts

    def set_checkpoint_interval(self, interval):
        assert interval >= 0
        self.activation_checkpoint_interval = interval

    def ckpt_prefix(self, checkpoints_path, tag):
        return os.path.join(checkpoints_path, str(tag))

    def ckpt_layer_path(self, ckpt_dir, local_layer_idx):
        idx = local_layer_idx + self._local_start
        suffix = self._grid._topo.get_rank_repr(rank=self.global_rank)
        return os.path.join(ckpt_dir, f"layer_{idx:02d}" + (f"-{suffix}" if suffix else "") + "-model_states.pt")

    def ckpt_layer_path_list(self, ckpt_dir, local_layer_idx):
        """Every model-slice file of one layer, sorted (one per tensor-parallel rank of the saving run)."""
        import glob
        idx = local_layer_idx + self._local_start
        return sorted(glob.glob(os.path.join(ckpt_dir, f"layer_{idx:02d}-*model_states.pt")))

    def _frozen_names(self, layer):
        return [n for n, p in layer.named_parameters() if not p.requires_grad]

    def save_state_dict(self, save_dir, checkpoint_engine, exclude_frozen_params=False):
        """One `layer_XX-model_YY-model_states.pt` per local layer (reference `runtime/pipe/module.py:567-598`): the
        files are indexed by GLOBAL layer number, so a checkpoint loads under any stage count. Replicas hold the same
        weights: replica 0 writes them all, or, with `checkpoint_parallel_write_pipeline`, each replica an even share
        (all 7 xGMI peers of a node writing at once instead of one)."""
        from ...checkpoint.utils import clone_tensors_for_torch_save
        dp_rank, dp_size = self._grid.data_parallel_id, self._grid.data_parallel_size
        n = len(self.forward_funcs)
        if self.checkpoint_parallel_write_pipeline:
            cuts = partition_uniform(n, dp_size)
            start, end = cuts[dp_rank], cuts[dp_rank + 1]
        elif dp_rank != 0:
            return
        else:
            start, end = 0, n
        checkpoint_engine.makedirs(save_dir, exist_ok=True)
        for i in range(start, end):
            layer = self.forward_funcs[i]
            if not hasattr(layer, "state_dict"):
                continue
            sd = layer.state_dict()
            if exclude_frozen_params:
                for name in self._frozen_names(layer):
                    del sd[name]
            checkpoint_engine.save(clone_tensors_for_torch_save(sd), self.ckpt_layer_path(save_dir, i))

    def load_state_dir(self, load_dir, checkpoint_engine, strict=True):
        """Inverse of `save_state_dict` (reference `runtime/pipe/module.py:600-625`): every local layer reads its
        file(s); a different tensor-parallel degree merges or splits them through the Megatron state-dict loader."""
        from ..state_dict_factory import SDLoaderFactory
        mp_rank = self._grid.get_slice_parallel_rank()
        mp_size = self._grid.get_slice_parallel_world_size()
        for i, layer in enumerate(self.forward_funcs):
            if not hasattr(layer, "load_state_dict"):
                continue
            files = self.ckpt_layer_path_list(load_dir, i)
            if not files:
                if strict:
                    raise FileNotFoundError(f"no checkpoint file for layer {i + self._local_start} in {load_dir}")
                continue
            loader = SDLoaderFactory.get_sd_loader(files, version=2.0, checkpoint_engine=checkpoint_engine)
            _, sd, _ = loader.load(mp_size, mp_rank, module_key=None, is_pipe_parallel=True)
            layer.load_state_dict(sd, strict=strict)
        self._synchronize_tied_weights()
