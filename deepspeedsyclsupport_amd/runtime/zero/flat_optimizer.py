"""Flat-group ZeRO engine: one implementation for "no ZeRO" (bf16/fp16/fp32 DP), ZeRO-1, ZeRO-2 and ZeRO-3.

Reference behaviour being reproduced: `runtime/zero/stage_1_and_2.py` (DeepSpeedZeroOptimizer: flatten, partition,
IPG buckets, reduce, all-gather after step), `runtime/zero/stage3.py` (DeepSpeedZeroOptimizer_Stage3: param shards,
reduce-scatter of grad buckets, sub-group stepping, Twin-Flow), `runtime/bf16_optimizer.py`,
`runtime/fp16/fused_optimizer.py`.

MI355X-first design (why it is not a port):
* A FLAT GROUP is a set of parameters laid out back-to-back in ONE buffer of `seg * dp` elements. Rank r owns the
  contiguous segment [r*seg, (r+1)*seg). Parameters are *views* into the gathered buffer, so
  - ZeRO-3 fetch = one `all_gather_into_tensor(full, shard)` and zero copies (the reference gathers per-param shards
    and unflattens with copies), released by swapping `p.data` back to an empty tensor;
  - gradient reduction = one `reduce_scatter_tensor(seg_out, grad_flat)` straight into the owner's segment
    (no interleave/pad copies as in the reference's `reduce_scatter_coalesced`);
  - ZeRO-1/2 post-step refresh = one in-place `all_gather_into_tensor` per group.
  With 288 GB of HBM per GPU the groups are big (per-module for ZeRO-3, `reduce_bucket_size` buckets otherwise),
  so every collective is a large xGMI transfer instead of many small ones.
* The optimizer works on per-optimizer-group fp32 master buffers made of "runs" (the intersection of a rank segment
  with one optimizer param group). The gfx950 fused Adam kernel updates master + moments and writes the bf16/fp16
  shard in the same pass (no separate cast), driven through the multi-tensor pointer table.
* Reduction runs on dedicated HIP streams (`rs_stream` for reduce-scatter / all-reduce, `ag_stream` for ZeRO-3
  prefetch all-gathers) and overlaps backward / forward compute; events order the hand-offs.
* ZeRO-Offload / Offload++ Twin-Flow: the first `ratio` fraction of each optimizer group's runs keep master and
  moments in pinned host memory and are stepped by the native CPU Adam CONCURRENTLY with the GPU part (the reference
  runs CPU and GPU sub-groups sequentially, `stage3.py:1976-1992`); D2H of grads and H2D of the bf16 result use
  non-blocking copies on a side stream.
"""
import math
import sys
import os
from collections import OrderedDict, defaultdict

import torch
import torch.nn as nn

from ... import comm as dist
from ...accelerator import get_accelerator
from ...checkpoint import constants as CK
from ...ops import native
from ...ops.adam.fused_adam import FusedAdam
from ...utils.logging import log_dist, logger
from .. import ZeROOptimizer
from ..fp16.loss_scaler import CreateLossScaler
from .config import ZeroStageEnum
from ...utils.nvtx import instrument_w_nvtx

ALIGN = 64  # elements: keeps every rank segment 128-B (bf16) aligned for 16-B vector access


def _ceil(a, b):
    return (a + b - 1) // b


def _pnumel(p):
    """Logical numel (zero.Init-partitioned params have empty .data and carry ds_numel)."""
    return p.ds_numel if hasattr(p, "ds_tensor") else p.numel()


class ZeroParamStatus:
    AVAILABLE = 1
    NOT_AVAILABLE = 2
    INFLIGHT = 3


class FlatGroup:
    """A set of parameters sharing one flat buffer and one collective."""

    def __init__(self, idx, params, dp, rank, partition, persistent, device, dtype, module=None, dp_group=None):
        self.idx = idx
        self.dp_group = dp_group    # reduction / partition group (DP, or expert-DP for MoE experts)
        self.reduce_dp = dp         # ranks that hold (a partition or a replica of) these params
        self.expert = False         # MoE expert parameters (set by the optimizer)
        self.params = list(params)
        self.module = module
        self.dtype = dtype
        self.device = device
        self.offsets, self.numels = [], []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            self.numels.append(_pnumel(p))
            off += _ceil(_pnumel(p), 8) * 8  # 16-B align each param view inside the buffer
        self.numel = off
        self.dp = dp if partition else 1
        self.rank = rank if partition else 0
        self.partition = partition
        self.seg = _ceil(max(self.numel, 1), self.dp * ALIGN) * ALIGN if partition else _ceil(max(self.numel, 1), ALIGN) * ALIGN
        self.padded = self.seg * self.dp
        self.persistent = persistent
        self.full = None          # gathered [padded] buffer (or None when released)
        self.shard = None         # [seg] owner shard (view of full for persistent groups)
        self.status = ZeroParamStatus.NOT_AVAILABLE
        self.ag_work = None
        self.ag_event = None
        self.grad_flat = None
        self.pending = 0
        self.reduced_this_pass = False
        self.runs = []            # (seg_lo, seg_hi, opt_group_idx, master_off, on_host)
        self.trace_pos = []
        self.frozen = False       # parameters the optimizer does not own: fetched / released, never reduced or stepped
        self.pieces = []

    @property
    def seg_lo(self):
        return self.rank * self.seg

    def param_seg_ranges(self, gidx_of_param):
        """Intersections of this rank's segment with each param: [(p_index, lo, hi)] in buffer coordinates."""
        lo, hi = self.seg_lo, self.seg_lo + self.seg
        out = []
        for i, p in enumerate(self.params):
            a, b = self.offsets[i], self.offsets[i] + self.numels[i]
            s, e = max(a, lo), min(b, hi)
            if s < e:
                out.append((i, s, e))
        return out


class FlatZeroOptimizer(ZeROOptimizer):
    """ZeRO stage 0/1/2/3 over flat groups. See module docstring."""

    def __init__(self, init_optimizer, module, ds_config, dp_group=None, stage=0, mpu=None, clip_grad=0.0,
                 dtype=torch.bfloat16, communication_data_type=None, zero_config=None, timers=None,
                 gradient_accumulation_steps=1, expert_params=None, sparse_params=None):
        self.optimizer = init_optimizer
        self.module = module
        self.sparse_params = set(sparse_params or ())  # ids of embedding weights reduced as sparse tensors
        self.sparse_reductions = 0
        self.stage = int(stage)
        self.zc = zero_config
        self.expert_grad_scaling = str(getattr(zero_config, "moe_expert_grad_scaling", "global") or "global")
        if self.expert_grad_scaling not in ("global", "expert_dp"):
            raise ValueError(f"moe_expert_grad_scaling must be 'global' or 'expert_dp', got {self.expert_grad_scaling}")
        self.safe_mode = bool(zero_config is not None and getattr(zero_config, "safe_mode", False))
        self.cfg = ds_config
        self.dtype = dtype
        self.clip_grad = clip_grad
        self.dp_group = dp_group
        self.dp = dist.get_world_size(dp_group)
        self.rank = dist.get_rank(dp_group)
        self.mpu = mpu
        self.timers = timers
        self.acc = get_accelerator()
        self.device = torch.device(self.acc.device_name(self.acc.current_device())) if self.acc.device_name() != "cpu" \
            else torch.device("cpu")
        # DS_ZERO_FORCE_PARTITION=1 runs the partitioned code path (all-gather / reduce-scatter on the comm streams,
        # shard pointing, qwZ/qgZ) even with one data-parallel rank: the single-GPU rehearsal of the multi-GPU path
        self.force_partition = os.environ.get("DS_ZERO_FORCE_PARTITION", "0") == "1"
        self.partition = self.stage >= 1 and (self.dp > 1 or self.force_partition)
        self.world = dist.get_world_size()
        self._setup_mics()
        self.comm_dtype = communication_data_type or dtype
        self.gas = gradient_accumulation_steps
        self.is_gradient_accumulation_boundary = True
        self.micro_step = 0
        self.global_steps = 0
        self.overflow = False
        self._global_grad_norm = None
        self.offload = False
        self.offload_ratio = 0.0
        self.offload_nvme = False
        self.off = None  # OffloadedState: host / NVMe resident optimizer state and its transfer pipelines
        oc = self.zc.offload_optimizer if self.zc is not None else None
        if oc is not None and _devname(oc.device) in ("cpu", "nvme"):
            self.offload = True
            self.offload_ratio = float(oc.ratio)
            self.offload_pin = bool(oc.pin_memory)
            self.offload_nvme = _devname(oc.device) == "nvme"
        self.nvme_swapper = None
        # split masters (bf16.split_master_weights): master bits = (bf16 weight << 16) + int16 residual
        self.split_master = bool(getattr(getattr(ds_config, "bf16_config", None), "split_master_weights", False))
        if self.split_master and dtype != torch.bfloat16:
            raise ValueError("bf16.split_master_weights needs bf16 training")
        # gradient scaling around the reduction (reference `runtime/engine.py:2331-2341`, passed to ZeRO at
        # `engine.py:1523,1595,1636`): prescale divides by the data-parallel size before the collective, otherwise
        # gradient_predivide_factor is applied before it and the remainder after
        self.prescale_gradients = bool(getattr(ds_config, "prescale_gradients", False))
        self.predivide = float(getattr(ds_config, "gradient_predivide_factor", 1.0) or 1.0)
        # ZeRO-Infinity parameter offload: non-persistent ZeRO-3 shards live in pinned host memory (cpu) or in
        # per-group files on NVMe mapped into the address space (nvme); every fetch streams them H2D on the
        # all-gather stream ahead of use (trace-driven prefetch), so HBM only holds the live working set.
        self.offload_param = False
        self.param_store = None
        op = self.zc.offload_param if self.zc is not None else None
        if self.stage == 3 and op is not None and _devname(op.device) in ("cpu", "nvme"):
            self.offload_param = True
            if _devname(op.device) == "nvme":
                from ..swap_tensor import ParamNvmeStore
                folder = os.path.join(op.nvme_path or "/tmp/ds_nvme_swap", "zero_stage_3", "params",
                                      f"rank{dist.get_rank()}")
                self.param_store = ParamNvmeStore(folder)
        # fp16 loss scaling
        fp16 = dtype == torch.float16
        self.loss_scaler = CreateLossScaler(dtype, getattr(ds_config, "loss_scale", 0) or 1.0,
                                            fp16 and getattr(ds_config, "loss_scale", 0) == 0,
                                            getattr(ds_config, "dynamic_loss_scale_args", None))
        self.dynamic_loss_scale = self.loss_scaler.dynamic
        # streams
        # side streams for the gradient reduce-scatter and the parameter all-gather: on unless the config says
        # `overlap_comm: false` in so many words (the key's unset default differs per stage in the reference; here
        # overlapping is the default for every stage)
        zc_set = getattr(self.zc, "model_fields_set", set()) if self.zc is not None else set()
        overlap = not ("overlap_comm" in zc_set and not self.zc.overlap_comm)
        self.rs_stream = self.acc.Stream() if self.device.type == "cuda" and overlap else None
        self.ag_stream = self.acc.Stream() if self.device.type == "cuda" and overlap else None
        # `reduce_scatter: false` (reference stage 1/2): all-reduce the whole bucket and keep the owner's slice
        self.use_reduce_scatter = bool(getattr(self.zc, "reduce_scatter", True)) if self.zc is not None else True
        self.ignore_unused = bool(getattr(self.zc, "ignore_unused_parameters", True)) if self.zc is not None else True
        self._fused_adam = isinstance(self.optimizer, FusedAdam) or getattr(self.optimizer, "_ds_flat_adam", False)
        self._build_groups()
        self._build_master()
        self._install_grad_hooks()
        self.coordinator = None
        if self.stage == 3 and (self.dp > 1 or self.offload_param or self.force_partition):
            from .coordinator import ParamCoordinator  # (also when only frozen groups are fetched)
            self.coordinator = ParamCoordinator(self, prefetch_bucket_size=self.zc.prefetch_bucket_size,
                                                max_live_parameters=self.zc.max_live_parameters,
                                                max_reuse_distance=self.zc.max_reuse_distance)
        log_dist(f"FlatZeroOptimizer: stage={self.stage} dp={self.dp} groups={len(self.groups)} "
                 f"params={sum(g.numel for g in self.groups) / 1e6:.1f}M partition={self.partition} "
                 f"offload={self.offload}(ratio={self.offload_ratio}) offload_param={self.offload_param} "
                 f"fused_adam={self._fused_adam}", ranks=[0])

    # ================================================================================ construction
    def _trainable_params_in_order(self):
        seen = set()
        out = []
        for og_idx, g in enumerate(self.optimizer.param_groups):
            for p in g["params"]:
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    out.append((p, og_idx))
        return out

    def _build_groups(self):
        plist = self._trainable_params_in_order()
        self.param_to_og = {id(p): og for p, og in plist}
        self.opt_params = [p for p, _ in plist]
        self.num_og = len(self.optimizer.param_groups)
        # reduction group per optimizer group: MoE expert groups (marked {'moe': True, 'name': ep_size_k}) reduce and
        # partition over their expert-data-parallel group, everything else over the (sequence x) data group
        self.og_dp_group = []
        for g in self.optimizer.param_groups:
            if g.get("moe", False):
                from ...parallel import groups as pgroups
                self.og_dp_group.append(pgroups._get_expert_data_parallel_group(g["name"]))
            else:
                self.og_dp_group.append(self.mics_shard_group or self.dp_group)
        groups = []
        if self.stage == 3:
            # one group per module that directly owns trainable params (fetch granularity = module), plus ONE
            # persistent group for every small param (< param_persistence_threshold): never released.
            fetched = self.dp > 1 or self.offload_param or self.force_partition  # gathered / streamed per module
            thr = self.zc.param_persistence_threshold if fetched else 0
            owned = set()
            persistent = []
            budget = int(getattr(self.zc, "model_persistence_threshold", sys.maxsize) or sys.maxsize)
            for name, m in self.module.named_modules():
                ps = [p for p in m.parameters(recurse=False) if id(p) in self.param_to_og and id(p) not in owned]
                if not ps:
                    continue
                for p in ps:
                    owned.add(id(p))
                for p in [p for p in ps if id(p) in self.sparse_params]:  # sparse-reduced weights: a group each
                    groups.append(dict(params=[p], persistent=not fetched, module=m, sparse=True))
                ps = [p for p in ps if id(p) not in self.sparse_params]
                small = []
                for p in ps:  # small parameters stay gathered while their total fits model_persistence_threshold
                    if _pnumel(p) < thr and _pnumel(p) <= budget:
                        small.append(p)
                        budget -= _pnumel(p)
                big = [p for p in ps if not any(p is q for q in small)]
                persistent.extend(small)
                if big:
                    big.sort(key=lambda p: self.param_to_og[id(p)])
                    groups.append(dict(params=big, persistent=not fetched, module=m))
            rest = [p for p in self.opt_params if id(p) not in owned]
            persistent.extend(rest)
            if persistent:
                persistent.sort(key=lambda p: self.param_to_og[id(p)])
                groups.append(dict(params=persistent, persistent=True, module=None))
        else:
            # buckets in REVERSE registration order (≈ backward order) so reduction of early buckets overlaps
            # the rest of backward; bucket size from reduce_bucket_size (default 5e8 elements ≈ 1 GB bf16)
            cap = int(self.zc.reduce_bucket_size) if self.zc is not None else int(5e8)
            cur, cur_n = [], 0
            for p in reversed(self.opt_params):
                if id(p) in self.sparse_params:
                    groups.append(dict(params=[p], persistent=True, module=None, sparse=True))
                    continue
                if cur and (cur_n + _pnumel(p) > cap or self.param_to_og[id(p)] != self.param_to_og[id(cur[-1])]):
                    groups.append(dict(params=cur, persistent=True, module=None))
                    cur, cur_n = [], 0
                cur.append(p)
                cur_n += _pnumel(p)
            if cur:
                groups.append(dict(params=cur, persistent=True, module=None))
        self.groups = []
        for i, d in enumerate(groups):
            og = self.param_to_og[id(d["params"][0])]
            pg = self.og_dp_group[og]
            gdp, grank = dist.get_world_size(pg), dist.get_rank(pg)
            multi = gdp > 1 or self.force_partition
            persistent = d["persistent"] or (not multi and not self.offload_param)
            g = FlatGroup(i, d["params"], gdp, grank, self.stage >= 1 and multi, persistent,
                          self.device, self.dtype, d["module"], dp_group=pg)
            g.expert = bool(self.optimizer.param_groups[og].get("moe", False))
            g.sparse = bool(d.get("sparse", False))
            self.groups.append(g)
        self._build_frozen_groups()
        self.param_group = {}
        import weakref
        ref = weakref.ref(self)
        for g in self.all_groups:
            for i, p in enumerate(g.params):
                self.param_group[id(p)] = (g, i)
                p._ds_zero_optimizer = ref  # lets utils.tensor_fragment.safe_get_* find the owner
        self._materialize_buffers()

    @property
    def all_groups(self):
        """Optimizer-owned groups followed by the frozen ones; `FlatGroup.idx` indexes this list."""
        return self.groups + self.frozen_groups

    def _build_frozen_groups(self):
        """ZeRO-3 partitions every module parameter, not only the trained ones (reference `stage3.py:419-470`,
        `parameter_offload.py:240-260`): with adapters on a frozen base model the frozen weights are most of the
        memory. Parameters the optimizer does not own (requires_grad=False, or simply not handed to it) get fetch
        groups of their own, one per owning module: partitioned, gathered before the module's forward / backward and
        released after, optionally homed on the host / NVMe with offload_param, but never reduced or stepped. Small
        ones (below the persistence threshold) and those of another dtype stay whole on every rank."""
        self.frozen_groups = []
        if self.stage != 3:
            return
        fetched = self.dp > 1 or self.offload_param or self.force_partition
        thr = self.zc.param_persistence_threshold if fetched else 0
        seen = set(self.param_to_og)
        base = len(self.groups)
        for name, m in self.module.named_modules():
            ps = [p for p in m.parameters(recurse=False) if id(p) not in seen]
            if not ps:
                continue
            seen.update(id(p) for p in ps)
            big = [p for p in ps if fetched and p.dtype == self.dtype and _pnumel(p) >= thr]
            for p in ps:
                if not any(p is q for q in big) and getattr(p, "ds_tensor", None) is not None \
                        and p.data.numel() != p.ds_numel:
                    # built partitioned under zero.Init but kept whole here
                    from .partition_parameters import gather_partitioned_param
                    p.data = gather_partitioned_param(p).clone()
                    del p.ds_tensor
            if not big:
                continue
            multi = self.dp > 1 or self.force_partition
            g = FlatGroup(base + len(self.frozen_groups), big, self.dp, self.rank, multi, False, self.device,
                          self.dtype, m, dp_group=self.dp_group)
            g.frozen = True
            self.frozen_groups.append(g)

    @torch.no_grad()
    def _materialize_buffers(self):
        """Move parameter data into flat buffers (full for persistent groups, shard-only for ZeRO-3)."""
        for g in self.all_groups:
            g._opt = self
            full = torch.zeros(g.padded, dtype=self.dtype, device=self.device)
            for i, p in enumerate(g.params):
                if getattr(p, "ds_tensor", None) is not None and p.data.numel() != p.ds_numel:
                    # built under zero.Init: re-gather this one parameter and regroup it into the flat layout
                    from .partition_parameters import gather_partitioned_param
                    src = gather_partitioned_param(p)
                else:
                    src = p.data
                full[g.offsets[i]:g.offsets[i] + g.numels[i]].copy_(src.reshape(-1))
                if hasattr(p, "ds_tensor"):
                    del p.ds_tensor
            if g.persistent:
                g.full = full
                g.shard = full[g.seg_lo:g.seg_lo + g.seg]
                self._point_params(g)
                g.status = ZeroParamStatus.AVAILABLE
            else:
                seg = full[g.seg_lo:g.seg_lo + g.seg]
                g.shard = self._offload_shard(g, seg) if self.offload_param else seg.clone()
                del full, seg
                g.full = None
                self._release_params(g)
            from .partition_parameters import _attach_api
            for i, p in enumerate(g.params):
                p.ds_numel = g.numels[i]
                p.ds_persist = g.persistent
                p.ds_group = g
                _attach_api(p)
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def _offload_shard(self, g, seg):
        """Host (pinned) or NVMe-backed home of an offloaded ZeRO-3 shard, initialised from `seg`."""
        if self.param_store is not None:
            return self.param_store.create(g.idx, seg)
        if self.device.type == "cuda":
            from ...ops.native import hip_ops
            host = hip_ops().alloc_pinned(g.seg, self.dtype)  # exact size (torch's pinned pool rounds to 2^k)
        else:
            host = torch.empty(g.seg, dtype=self.dtype)
        host.copy_(seg)
        return host

    def _point_params(self, g):
        for i, p in enumerate(g.params):
            shape = getattr(p, "ds_shape", None) or p.shape
            if not hasattr(p, "ds_shape"):
                p.ds_shape = shape
            p.data = g.full[g.offsets[i]:g.offsets[i] + g.numels[i]].view(shape)
            p.ds_status = ZeroParamStatus.AVAILABLE

    def _release_params(self, g):
        for i, p in enumerate(g.params):
            if not hasattr(p, "ds_shape"):
                p.ds_shape = p.shape
            p.ds_numel = g.numels[i]
            p.data = torch.empty(0, dtype=self.dtype, device=self.device)
            p.ds_status = ZeroParamStatus.NOT_AVAILABLE
        g.status = ZeroParamStatus.NOT_AVAILABLE

    @torch.no_grad()
    def _build_master(self):
        """Optimizer-state layout: per optimizer group the local elements are concatenated "runs" (rank-segment ∩
        optimizer group). The LAST `ratio` of each group's elements (in forward order) is offloaded — those layers'
        gradients are final first in backward, so their copies down overlap the rest of backward, and their weights
        are needed last by the next forward, so the host update overlaps it — and handed to `OffloadedState`; the
        rest keeps fp32 master (or int16 residuals with split masters) and moments on the device."""
        og_len = [0] * self.num_og
        run_specs = []
        for g in self.groups:
            ranges = g.param_seg_ranges(None)
            runs = []
            for (i, s, e) in ranges:
                og = self.param_to_og[id(g.params[i])]
                if runs and runs[-1][2] == og:
                    runs[-1][1] = e  # contiguous or separated only by alignment padding (zero, stays zero)
                else:
                    runs.append([s, e, og])
            for s, e, og in runs:
                run_specs.append((g, s, e, og))
                og_len[og] += e - s
        if self.split_master and not self._fused_adam:
            raise ValueError("bf16.split_master_weights is implemented for Adam / AdamW only")
        boundary = [l - int(l * self.offload_ratio) if self.offload else l for l in og_len]
        pos = [0] * self.num_og
        dev_len = [0] * self.num_og
        host_len = [0] * self.num_og
        split_specs = []
        for g, s, e, og in run_specs:
            # a run straddling the device/host boundary is cut there (at a 64-element multiple of its start)
            cut = s + (boundary[og] - pos[og]) // ALIGN * ALIGN
            pos[og] += e - s
            if self.offload and s < cut < e:
                split_specs += [(g, s, cut, og, False), (g, cut, e, og, True)]
            else:
                split_specs.append((g, s, e, og, self.offload and cut <= s))
        for g, s, e, og, on_host in split_specs:
            n = e - s
            if on_host:
                moff = host_len[og]
                host_len[og] += n
            else:
                moff = dev_len[og]
                dev_len[og] += n
            g.runs.append((s - g.seg_lo, e - g.seg_lo, og, moff, on_host))
        self.master = []
        self.grad_acc = []
        mdt = torch.int16 if self.split_master else torch.float32
        for og in range(self.num_og):
            self.master.append(torch.zeros(dev_len[og], dtype=mdt, device=self.device))
            self.grad_acc.append(None)  # fp32 accumulator, allocated only when a path needs it
        for g in self.groups:
            g.pieces = []    # offloaded runs of this group (OffloadedState pieces)
            g.host_map = {}
            for (s, e, og, moff, on_host) in g.runs:
                if not on_host and not self.split_master:
                    self.master[og][moff:moff + e - s].copy_(g.shard[s:e])
        if self.offload and any(host_len):
            self._build_offload(host_len)
        # hand the optimizer one flat parameter per group (its param_groups / lr schedule stay authoritative); with
        # split masters there is no fp32 tensor to hand over, an empty placeholder keys the moments instead
        self.fp32_flat = []
        for og, group in enumerate(self.optimizer.param_groups):
            data = torch.empty(0, dtype=torch.float32, device=self.device) if self.split_master else self.master[og]
            mp = nn.Parameter(data, requires_grad=False)
            self.fp32_flat.append(mp)
            group["params"] = [mp]

    def _build_offload(self, host_len):
        from .offload import OffloadedState
        oc = self.zc.offload_optimizer
        pin = self.device.type == "cuda" and getattr(self, "offload_pin", True)
        resident = list(host_len)
        if self.offload_nvme:
            budget = int(getattr(oc, "max_in_cpu", 0) or 0)
            for og in range(self.num_og):
                resident[og] = min(host_len[og], budget)
                budget -= resident[og]
            from ..swap_tensor import OptimizerStateSwapper
            path = oc.nvme_path or "/tmp/ds_nvme_swap"
            folder = os.path.join(path, f"zero_stage_{self.stage}", "optimizer", f"rank{dist.get_rank()}")
            # ZeRO-Infinity: master AND moments of the NVMe tail live in files, streamed in sub_group_size chunks
            # (reference partitioned_optimizer_swapper: fp32 params + optimizer states)
            chunk = int(min(getattr(self.zc, "sub_group_size", 64 * 2**20) or 64 * 2**20, 64 * 2**20))
            self.nvme_swapper = OptimizerStateSwapper(self.cfg.aio_config, folder, chunk_numel=max(chunk, 1),
                                                      pin=self.device.type == "cuda", with_master=True,
                                                      master_dtype=torch.int16 if self.split_master
                                                      else torch.float32)
        self.off = OffloadedState(self, host_len, resident, self.split_master, pin, self.nvme_swapper,
                                  overlap_forward=bool(getattr(oc, "overlap_forward", False)))
        for g in self.groups:
            for (s, e, og, moff, on_host) in g.runs:
                if on_host:
                    g.pieces.append(self.off.add_piece(og, moff, e - s, g, s))
        self.off.finalize()
        for p in self.off.all_pieces:
            self.off.init_master(p)
        for og in range(self.num_og):
            if host_len[og] > resident[og]:
                self.nvme_swapper.register(og, host_len[og] - resident[og], master_init=self.off.nvme_master_init(og))
        # LOCAL-mode staging map: param index -> [(piece, offset in piece, offset in param, numel)]
        for g in self.groups:
            g.host_map = {}
            for piece in g.pieces:
                lo, hi = g.seg_lo + piece.s, g.seg_lo + piece.s + piece.n
                for i in range(len(g.params)):
                    a, n = g.offsets[i], g.numels[i]
                    x0, x1 = max(a, lo), min(a + n, hi)
                    if x0 < x1:
                        g.host_map.setdefault(i, []).append((piece, x0 - lo, x0 - a, x1 - x0))
        if self.off.overlap_forward:
            self._install_offload_waits()

    def _install_offload_waits(self):
        """overlap_forward: each module owning offloaded weights waits for its own copy before its forward."""
        self._offload_wait_hooks = []
        for g in self.groups:
            if g.pieces and g.module is not None and g.persistent:  # fetched groups wait inside the coordinator
                self._offload_wait_hooks.append(
                    g.module.register_forward_pre_hook(lambda m, a, g=g: self.off.wait_group(g)))

    def offload_pre_forward(self):
        """Engine hook at the start of forward: groups without an owning module wait here (overlap_forward)."""
        if self.off is not None and self.off.overlap_forward:
            for g in self.groups:
                if g.pieces and g.module is None and g.persistent:
                    self.off.wait_group(g)

    def join_offload(self):
        """Block until the host partition's step has finished and its weights are back in the shards."""
        if self.off is not None:
            self.off.wait()

    def _ensure_grad_acc(self, og):
        if self.grad_acc[og] is None:
            self.grad_acc[og] = torch.zeros(self.master[og].numel(), dtype=torch.float32, device=self.device)
        return self.grad_acc[og]

    # ================================================================================ gradient path
    # Per group the gradient lives in one of three places (chosen for the fewest HBM passes):
    #   LOCAL  (no peer holds these params: dp == 1 for the group): autograd's own p.grad tensors feed the fused Adam
    #          directly — no flat buffer, no copy, no zero-fill; accumulation across micro-steps is autograd's.
    #   PRESET (ZeRO-0/1 with peers): p.grad are views into a persistent flat bf16 buffer that autograd accumulates into
    #          in place; one reduce-scatter/all-reduce per group at the accumulation boundary; its output feeds Adam.
    #   COPY   (ZeRO-2/3 with peers): the grad hook copies p.grad into a bucket and frees it; the bucket is reduced as
    #          soon as the group is complete (overlapping the rest of backward); with GAS == 1 the reduced bf16
    #          segment feeds Adam directly, with GAS > 1 it is accumulated into an fp32 partition.
    LOCAL, PRESET, COPY = 0, 1, 2

    def _mode(self, g):
        if g.reduce_dp == 1 and not self.force_partition:
            return self.LOCAL
        return self.PRESET if self.stage <= 1 else self.COPY

    def _install_grad_hooks(self):
        self._hooks = []
        for g in self.groups:
            g.mode = self._mode(g)
            g.red_out = None
            g._acc_valid = False
            if g.mode == self.PRESET:
                g.grad_flat = torch.zeros(g.padded, dtype=self.dtype, device=self.device)
                self._point_grads(g)
        # `grad_hooks: false` (reference `zero/config.py: grad_hooks`, stages 1/2): no per-parameter hooks fire
        # inside autograd; the whole pass is folded into the flat buffers and reduced in `backward_epilogue`
        self.grad_hooks = bool(getattr(self.zc, "grad_hooks", True)) if self.zc is not None else True
        if not self.grad_hooks:
            if self.stage == 3:
                raise ValueError("zero_optimization.grad_hooks=false is for stages 0-2: stage 3 releases gathered "
                                 "parameters from the gradient hooks")
            return
        for p in self.opt_params:
            g, _ = self.param_group[id(p)]
            if g.mode != self.LOCAL or self.coordinator_needed() or g.pieces:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._grad_ready_hook))

    def coordinator_needed(self):
        return self.stage == 3 and any(not g.persistent for g in self.all_groups)

    def _point_grads(self, g):
        for i, p in enumerate(g.params):
            p.grad = g.grad_flat[g.offsets[i]:g.offsets[i] + g.numels[i]].view(p.ds_shape)

    def _begin_pass(self):
        for g in self.groups:
            g.pending = len(g.params)
            g.reduced_this_pass = False

    def _grad_ready_hook(self, p):
        g, i = self.param_group[id(p)]
        if p.grad is not None and p.grad.is_sparse:
            p.grad = p.grad.to_dense()  # nn.Embedding(sparse=True): the flat buffers and the fused Adam are dense
        if g.mode == self.PRESET:
            view = g.grad_flat[g.offsets[i]:g.offsets[i] + g.numels[i]]
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                # p.grad was reset (e.g. module.zero_grad(set_to_none=True)): fold it back into the flat buffer
                if p.grad is not None:
                    view.add_(p.grad.reshape(-1))
                p.grad = view.view(p.ds_shape)
        elif g.mode == self.COPY:
            if g.grad_flat is None:
                g.grad_flat = torch.zeros(g.padded, dtype=self.dtype, device=self.device)
            g.grad_flat[g.offsets[i]:g.offsets[i] + g.numels[i]].copy_(p.grad.reshape(-1))
            p.grad = None
        elif g.pieces and self.is_gradient_accumulation_boundary and i in g.host_map:
            # LOCAL + offload: this parameter's (accumulated) gradient is final; send it down and free it
            flat = p.grad.reshape(-1)
            for (piece, poff, lo, n) in g.host_map[i]:
                self.off.stage_grad(piece, flat[lo:lo + n], 1.0 / self._div(g), off=poff)
            if sum(n for (_, _, _, n) in g.host_map[i]) == g.numels[i]:
                p.grad = None  # (a parameter cut by the device/host boundary keeps its gradient for the device part)
        if self.safe_mode and g.pending <= 0:
            from .utils import ZeRORuntimeException
            raise ZeRORuntimeException(f"fetch group {g.idx}: more gradients than parameters in one backward pass "
                                       "(a parameter's gradient was produced twice)")
        g.pending -= 1
        if g.pending == 0 and g.mode != self.LOCAL and self._should_reduce_now():
            self._reduce_group(g)
        if self.coordinator is not None and g.pending == 0 and not g.persistent:
            self.coordinator.release_after_backward(g)

    def _should_reduce_now(self):
        # ZeRO-0/1 accumulate locally and reduce only at the accumulation boundary
        return self.is_gradient_accumulation_boundary or self.stage >= 2

    def _local_grads(self):
        f = getattr(self.optimizer, "skip_grad_allreduce", None)
        return bool(f()) if f is not None else False

    def _div(self, g=None):
        # gradient = mean over the GLOBAL batch (dense DP size), for expert groups too by default; with
        # zero_optimization.moe_expert_grad_scaling = "expert_dp" expert grads are averaged over the expert-DP group
        # only (an ep-times larger scale: the reference's `stage_1_and_2.py` average_tensor numerics)
        if self._local_grads():
            return 1.0
        if g is not None and g.expert and self.expert_grad_scaling == "expert_dp":
            return float(g.reduce_dp)
        return float(self.dp)

    def _pre_factor(self, g=None):
        """Factor applied to the gradients BEFORE the collective (the rest of 1/div is applied after it, folded into
        the optimizer's gradient scale): 1/div with prescale_gradients (or fp16 communication, where the sum could
        overflow), else 1/gradient_predivide_factor."""
        div = self._div(g)
        if div <= 1:
            return 1.0
        if self.prescale_gradients or self.comm_dtype == torch.float16:
            return 1.0 / div
        return 1.0 / self.predivide if self.predivide != 1.0 else 1.0

    @instrument_w_nvtx
    def _reduce_group(self, g):
        if g.reduced_this_pass:
            return
        g.reduced_this_pass = True
        if self.safe_mode and not self._local_grads():
            from .utils import assert_ints_same_as_other_ranks
            assert_ints_same_as_other_ranks([g.idx, g.padded, int(g.partition)], g.dp_group,
                                            "gradient reduction (group id, numel, partitioned)")
        src = g.grad_flat
        compute = self.acc.current_stream() if self.rs_stream is not None else None
        ctx = self.acc.stream(self.rs_stream) if self.rs_stream is not None else _nullctx()
        if self.rs_stream is not None:
            self.rs_stream.wait_stream(compute)
        with ctx:
            comm = src if src.dtype == self.comm_dtype else src.to(self.comm_dtype)
            pre = self._pre_factor(g)
            if pre != 1.0:
                comm.mul_(pre)
            if self._local_grads():
                out = comm  # a communication-compressed optimizer (1-bit Adam/LAMB, 0/1 Adam) averages on its own
            elif getattr(g, "sparse", False) and g.reduce_dp > 1:
                comm = self._sparse_reduce(g, comm)
                out = comm[g.seg_lo:g.seg_lo + g.seg]
            elif g.partition and not self.use_reduce_scatter and self.mics_replica_group is None:
                dist.all_reduce(comm, group=g.dp_group)
                out = comm[g.seg_lo:g.seg_lo + g.seg]
            elif g.partition:
                out = torch.empty(g.seg, dtype=comm.dtype, device=comm.device)
                if self.zc is not None and self.zc.zero_quantized_gradients:
                    # qgZ: int8 all-to-all + fused dequant-reduce; two levels (inside the node, then between
                    # nodes) when the group spans several nodes
                    from .zeropp import qgz_groups, quantized_reduce_scatter, quantized_reduce_scatter_2level
                    if not hasattr(self, "_qgz_levels"):
                        self._qgz_levels = qgz_groups(g.dp_group)
                    if self._qgz_levels is not None:
                        quantized_reduce_scatter_2level(out, comm, *self._qgz_levels)
                    else:
                        quantized_reduce_scatter(out, comm, g.dp_group)
                else:
                    dist.reduce_scatter_tensor(out, comm, group=g.dp_group)
                if self.mics_replica_group is not None and g.dp_group is self.mics_shard_group:
                    dist.all_reduce(out, group=self.mics_replica_group)
            else:
                dist.all_reduce(comm, group=g.dp_group)
                out = comm[g.seg_lo:g.seg_lo + g.seg]
            accumulate = g.mode == self.COPY and self.gas > 1
            for piece in g.pieces:  # offloaded runs: the reduced segment goes down to the host now
                self.off.stage_grad(piece, out[piece.s:piece.s + piece.n], self._alpha(g), accumulate=accumulate)
            if accumulate:
                self._accumulate_runs(g, out, self._alpha(g))
            elif any(not r[4] for r in g.runs):
                g.red_out = out
            if g.mode == self.COPY:
                if self.rs_stream is not None:
                    src.record_stream(self.rs_stream)
                g.grad_flat = None

    def _sparse_reduce(self, g, flat):
        """Sum a row-sparse embedding gradient over the group by all-gathering (row indices, rows) (reference
        `runtime/engine.py:2462-2518` sparse_allreduce) and scatter-adding them back into the dense flat buffer."""
        from ..sparse_tensor import SparseTensor, sparse_allreduce
        p = g.params[0]
        rows = p.ds_shape[0]
        dense = flat[:g.numels[0]].view(rows, g.numels[0] // rows)
        st = sparse_allreduce(SparseTensor(dense), group=g.dp_group, average=False)
        flat.zero_()
        dense.index_add_(0, st.indices, st.values)
        self.sparse_reductions += 1
        return flat

    def _alpha(self, g=None):
        """Factor still owed to the reduced gradient: 1 / (div * pre_factor)."""
        div = self._div(g)
        return 1.0 if div == 1 else 1.0 / (div * self._pre_factor(g))

    def _accumulate_runs(self, g, seg_grad, alpha):
        first = not g._acc_valid
        for (s, e, og, moff, on_host) in g.runs:
            if on_host:
                continue  # accumulated on the host by OffloadedState
            src = seg_grad[s:e]
            dst = self._ensure_grad_acc(og)[moff:moff + e - s]
            if first:
                torch.mul(src, alpha, out=dst) if alpha != 1.0 else dst.copy_(src)
            else:
                dst.add_(src, alpha=alpha)
        g._acc_valid = True

    def backward_prologue(self):
        self._begin_pass()
        if self.coordinator is not None:
            self.coordinator.begin_backward()

    def backward(self, loss, retain_graph=False):
        self.backward_prologue()
        if self.dtype == torch.float16:
            self.loss_scaler.backward(loss.float(), retain_graph=retain_graph)
        else:
            loss.backward(retain_graph=retain_graph)
        self.backward_epilogue()

    @instrument_w_nvtx
    def backward_epilogue(self):
        """Flush groups whose params got no grad this pass (unused params count as zero) and join streams."""
        if not self.grad_hooks:
            for p in reversed(self.opt_params):
                g, _ = self.param_group[id(p)]
                if p.grad is not None and (g.mode != self.LOCAL or g.pieces):
                    self._grad_ready_hook(p)
        if not self.ignore_unused:
            names = None
            for g in self.groups:
                if g.pending > 0:
                    if names is None:
                        names = {id(p): n for n, p in self.module.named_parameters()}
                    missing = [names.get(id(p), "?") for p in g.params if p.grad is None and g.mode == self.LOCAL] \
                        or [names.get(id(p), "?") for p in g.params][:g.pending]
                    from .utils import ZeRORuntimeException
                    raise ZeRORuntimeException(
                        f"{g.pending} parameter(s) of fetch group {g.idx} received no gradient in this backward pass "
                        f"(e.g. {missing[:3]}) and zero_optimization.ignore_unused_parameters is false")
        if self._should_reduce_now():
            for g in self.groups:
                if g.mode != self.LOCAL and not g.reduced_this_pass:
                    if g.grad_flat is None:
                        g.grad_flat = torch.zeros(g.padded, dtype=self.dtype, device=self.device)
                    self._reduce_group(g)
        if self.rs_stream is not None:
            self.acc.current_stream().wait_stream(self.rs_stream)
        if self.coordinator is not None:
            self.coordinator.end_backward()
        self.micro_step += 1

    def reduce_gradients(self, pipeline_parallel=False):
        """Boundary reduction issued explicitly (pipeline engine: after tied-weight gradients were summed)."""
        self.is_gradient_accumulation_boundary = True
        for g in self.groups:
            if g.mode != self.LOCAL:
                g.reduced_this_pass = False
                if g.grad_flat is None:
                    g.grad_flat = torch.zeros(g.padded, dtype=self.dtype, device=self.device)
                self._reduce_group(g)
        if self.rs_stream is not None:
            self.acc.current_stream().wait_stream(self.rs_stream)

    # ================================================================================ step
    def _unscale_factor(self):
        return 1.0 / self.loss_scaler.loss_scale

    def _og_replicas(self, og):
        """Ranks holding an identical copy of each element of this og's local master (1 when partitioned)."""
        pg = self.og_dp_group[og]
        n = dist.get_world_size(pg)
        base = 1 if (self.stage >= 1 and n > 1) else n
        if self.mics_shard_group is not None and pg is self.mics_shard_group:
            base *= self.mics_replicas
        return base

    def partition_count(self):
        if not self.partition:
            return 1
        return self.dp // self.mics_replicas

    # ================================================================================ MiCS
    def _setup_mics(self):
        """MiCS (reference `runtime/zero/mics.py`): partition dense params inside groups of `mics_shard_size`
        consecutive ranks (one xGMI node) and replicate across groups; gradients reduce-scatter inside the shard
        group, then all-reduce across replicas (the only inter-group traffic)."""
        self.mics_shard_group = None
        self.mics_replica_group = None
        self.mics_replicas = 1
        self.mics_hier = None
        S = int(getattr(self.zc, "mics_shard_size", -1) or -1) if self.zc is not None else -1
        if S <= 1 or S >= self.dp or self.stage < 1:
            return
        from .mics_utils import create_mics_comm_groups
        ranks = dist.get_all_ranks_from_group(self.dp_group) if self.dp != self.world else list(range(self.world))
        cg = create_mics_comm_groups(S, self.dp_group, bool(getattr(self.zc, "mics_hierarchical_params_gather",
                                                                    False)), ranks=ranks)
        self.mics_groups = cg
        self.mics_shard_group, self.mics_replica_group = cg.param_shard_group, cg.param_repli_group
        self.mics_replicas = cg.param_repli_size
        # a shard group that spans nodes gathers its parameters in two levels
        if cg.param_intra_node_group is not None:
            self.mics_hier = (cg.param_intra_node_group, cg.param_inter_node_shard_group)

    def _grad_items(self):
        """[(og, moff, n, grad_1d, lp_1d, scale)] covering every DEVICE-resident master element that has a gradient
        (offloaded elements were staged to the host during backward)."""
        items = []
        for g in self.groups:
            alpha, div = self._alpha(g), self._div(g)
            for (s, e, og, moff, on_host) in g.runs:
                if on_host:
                    continue
                if g.mode == self.LOCAL:
                    for i, p in enumerate(g.params):
                        a, n = g.offsets[i], g.numels[i]
                        lo, hi = max(a, g.seg_lo + s), min(a + n, g.seg_lo + e)
                        if lo >= hi or p.grad is None:
                            continue
                        if p.grad.is_sparse:
                            p.grad = p.grad.to_dense()
                        gr = p.grad.reshape(-1)[lo - a:hi - a]
                        items.append((og, moff + lo - g.seg_lo - s, hi - lo, gr, g.shard[lo - g.seg_lo:hi - g.seg_lo],
                                      1.0 / div))
                elif g._acc_valid:
                    items.append((og, moff, e - s, self.grad_acc[og][moff:moff + e - s], g.shard[s:e], 1.0))
                elif g.red_out is not None:
                    items.append((og, moff, e - s, g.red_out[s:e], g.shard[s:e], alpha))
        return items

    @torch.no_grad()
    def _global_norm_sq(self, items):
        """Squared global grad norm: each rank sums its unique elements (replicas divided out) and ONE all-reduce over
        the world adds dense DP partitions, expert partitions and tensor-parallel shards alike. Gradients already
        staged to the host contribute the sums taken on their way down."""
        classes = defaultdict(list)
        for (og, moff, n, gr, lp, scale) in items:
            classes[(og, scale, gr.device.type)].append(gr)
        sq = torch.zeros((), dtype=torch.float32, device=self.device)
        for (og, scale, devtype), ts in classes.items():
            if devtype == "cuda":
                s = native.hip_ops().sumsq_multi([t.contiguous() for t in ts])
            else:
                s = sum((t.float().pow(2).sum() for t in ts), torch.zeros(())).to(self.device)
            sq = sq + s * (scale * scale) / self._og_replicas(og)
        if self.off is not None:
            for og, s in self.off.staged_norm_sq().items():
                s = s.to(self.device) if torch.is_tensor(s) else torch.tensor(float(s), device=self.device)
                sq = sq + s.float() / self._og_replicas(og)
        if self.world > 1:
            dist.all_reduce(sq)
        return sq

    @torch.no_grad()
    @instrument_w_nvtx
    def step(self, closure=None, lr_kwargs=None):
        """Optimizer step at the accumulation boundary (the engine only calls it there)."""
        items = self._grad_items()
        scale = self._unscale_factor()
        norm = self._global_norm_sq(items).sqrt() * scale
        norm_f = float(norm)  # the one device->host sync per step (overflow / clipping decisions)
        self._global_grad_norm = norm_f
        overflow = not math.isfinite(norm_f)
        self.overflow = overflow
        if self.dtype == torch.float16 or self.loss_scaler.dynamic:
            self.loss_scaler.update_scale(overflow)
        if overflow:
            log_dist(f"Overflow detected. Skipping step. Attempted loss scale: {1 / scale}, reducing to "
                     f"{self.loss_scaler.loss_scale}", ranks=[0])
            if self.off is not None:
                self.off.discard()
            self._zero_grad_buffers()
            return
        clip = 1.0
        if self.clip_grad and self.clip_grad > 0 and norm_f > self.clip_grad:
            clip = self.clip_grad / (norm_f + 1e-6)
        grad_scale = scale * clip
        if self.off is not None:
            # Twin-Flow: the host partition is stepped by the offload worker (CPU Adam + weight copies on the h2d
            # stream) while this thread launches the device optimizer
            self.off.step(grad_scale, self._host_hyper())
        self._device_step(items, grad_scale)
        if self.off is not None and (not self.off.overlap_forward or
                                     any(g.partition and g.persistent and g.pieces for g in self.groups)):
            self.off.wait()  # (persistent partitioned groups re-gather their shards right below)
        self._post_step_gather()
        self._zero_grad_buffers()
        self.global_steps += 1

    def _host_hyper(self):
        if not self._fused_adam:
            raise NotImplementedError("optimizer offload steps the host partition with the native CPU Adam: use "
                                      "Adam / AdamW (got " + type(self.optimizer).__name__ + ")")
        adamw = bool(getattr(self.optimizer, "adam_w_mode", True))
        return [dict(lr=g["lr"], betas=tuple(g["betas"]), eps=g["eps"], weight_decay=g["weight_decay"],
                     bias_correction=g.get("bias_correction", True), adamw=adamw)
                for g in self.optimizer.param_groups]

    def _moments(self, og):
        """Device-resident Adam state of og (created on first use), keyed by the group's flat parameter."""
        st = self.optimizer.state[self.fp32_flat[og]]
        if len(st) == 0:
            n = self.master[og].numel()
            st["step"] = 0
            st["exp_avg"] = torch.zeros(n, dtype=torch.float32, device=self.device)
            st["exp_avg_sq"] = torch.zeros(n, dtype=torch.float32, device=self.device)
        return st

    @instrument_w_nvtx
    def _device_step(self, items, grad_scale):
        adamw = bool(getattr(self.optimizer, "adam_w_mode", True))
        if self._fused_adam:
            by_og = defaultdict(list)
            for it in items:
                by_og[it[0]].append(it)
            for og, group in enumerate(self.optimizer.param_groups):
                master = self.master[og]
                st = self._moments(og)
                st["step"] += 1
                if master.numel() == 0 or not by_og.get(og):
                    continue
                b1, b2 = group["betas"]
                step = st["step"]
                bc = group.get("bias_correction", True)
                bc1 = 1 - b1**step if bc else 1.0
                bc2 = 1 - b2**step if bc else 1.0
                # one multi-tensor launch per (grad dtype, grad scale) class
                classes = defaultdict(list)
                for (_, moff, n, gr, lp, s) in by_og[og]:
                    classes[(gr.dtype, s)].append((moff, n, gr, lp))
                for (gdt, s), lst in classes.items():
                    ps = [master[moff:moff + n] for moff, n, _, _ in lst]
                    ms = [st["exp_avg"][moff:moff + n] for moff, n, _, _ in lst]
                    vs = [st["exp_avg_sq"][moff:moff + n] for moff, n, _, _ in lst]
                    gs = [gr for _, _, gr, _ in lst]
                    lps = [lp for _, _, _, lp in lst]
                    if master.is_cuda:
                        # offloaded shards: the kernel works on a device copy, streamed back to the host home after
                        back = [(i, lp) for i, lp in enumerate(lps) if not lp.is_cuda]
                        for i, lp in back:
                            lps[i] = lp.to(master.device, non_blocking=True) if self.split_master else \
                                torch.empty(lp.numel(), dtype=lp.dtype, device=master.device)
                        if self.split_master:
                            native.hip_ops().adam_multi_split(ps, ms, vs, gs, lps, group["lr"], b1, b2, group["eps"],
                                                              group["weight_decay"], bc1, bc2, grad_scale * s, adamw)
                        else:
                            native.hip_ops().adam_multi(ps, ms, vs, gs, lps, group["lr"], b1, b2, group["eps"],
                                                        group["weight_decay"], bc1, bc2, grad_scale * s, adamw)
                        for i, lp in back:
                            lp.copy_(lps[i], non_blocking=lp.is_pinned())
                    else:
                        # host flats (CPU accelerator / gloo): the native AVX-512 Adam (csrc/cpu/cpu_optim.cpp)
                        cpu = native.cpu_ops()
                        for p_, m_, v_, g_, lp_ in zip(ps, ms, vs, gs, lps):
                            if self.split_master:
                                hi = lp_.contiguous()
                                cpu.cpu_adam_update_split(p_, m_, v_, g_.contiguous(), hi, hi, step, group["lr"], b1,
                                                          b2, group["eps"], group["weight_decay"], bc, adamw,
                                                          grad_scale * s)
                                if hi.data_ptr() != lp_.data_ptr():
                                    lp_.copy_(hi)
                            else:
                                cpu.cpu_adam_update(p_, m_, v_, g_.contiguous(), lp_, step, group["lr"], b1, b2,
                                                    group["eps"], group["weight_decay"], bc, adamw, grad_scale * s)
        else:
            # generic torch optimizer over the fp32 flats: materialise scaled fp32 grads, step, copy to shards
            for og in range(self.num_og):
                self._ensure_grad_acc(og)
            for (og, moff, n, gr, lp, s) in items:
                dst = self.grad_acc[og][moff:moff + n]
                if dst.data_ptr() == gr.data_ptr():
                    dst.mul_(grad_scale)
                else:
                    torch.mul(gr, grad_scale * s, out=dst) if gr.dtype == torch.float32 else \
                        dst.copy_(gr).mul_(grad_scale * s)
            for og in range(self.num_og):
                self.fp32_flat[og].grad = self.grad_acc[og]
            self.optimizer.step()
            for (og, moff, n, gr, lp, s) in items:
                lp.copy_(self.master[og][moff:moff + n])

    def _post_step_gather(self):
        """Refresh full params of persistent groups from the updated shards (ZeRO-1/2, ZeRO-3 persistent)."""
        no_allgather = bool(getattr(self.cfg, "disable_allgather", False))
        for g in self.groups:
            if g.partition and g.persistent and g.full is not None:
                if not no_allgather:
                    dist.all_gather_into_tensor(g.full, g.shard, group=g.dp_group)
                    continue
                # `disable_allgather` (reference `runtime/config.py:270`): every owner broadcasts its segment instead
                # (for fabrics or debug sessions where the all-gather is the suspect); same bytes, dp launches
                for r in range(g.dp):
                    piece = g.full[r * g.seg:(r + 1) * g.seg]
                    if r == g.rank and piece.data_ptr() != g.shard.data_ptr():
                        piece.copy_(g.shard)
                    dist.broadcast(piece, dist.get_global_rank(g.dp_group, r), group=g.dp_group)

    def _zero_grad_buffers(self):
        for g in self.groups:
            g._acc_valid = False
            g.red_out = None
            if g.mode == self.PRESET and g.grad_flat is not None:
                g.grad_flat.zero_()
            elif g.mode == self.LOCAL:
                for p in g.params:
                    p.grad = None
        self.micro_step = 0

    def zero_grad(self, set_to_none=True):
        # gradients are owned by the optimizer between backward and step (see gradient-path comment)
        pass

    # ================================================================================ accessors / compat
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def loss_scale(self):
        return self.loss_scaler.loss_scale

    @property
    def cur_scale(self):
        return self.loss_scaler.loss_scale

    def get_global_grad_norm(self):
        return self._global_grad_norm

    def scale_if_loss(self, loss):
        return loss * self.loss_scaler.loss_scale if self.dtype == torch.float16 else loss

    # ---------------------------------------------------------------- per-parameter views of flat fp32 state
    # Two primitives address optimizer state by (group, run, segment range): `_run_read` returns fp32 values on the
    # compute device, `_run_write` stores them. `key` is "fp32" (master), "exp_avg" or "exp_avg_sq". They hide where
    # the state lives (device flat, host DRAM, NVMe) and how the master is stored (fp32, or bf16 weight + residual).
    def _run_read(self, g, run, key, a, b):
        s, e, og, moff, on_host = run
        lo = moff + a - s
        if on_host:
            if key == "fp32" and self.split_master:
                res = self.off.read_state(og, "residual", lo, lo + b - a).to(self.device)
                return _split_join(g.shard[a:b].to(self.device), res)
            t = self.off.read_state(og, key, lo, lo + b - a)
            return None if t is None else t.to(self.device, torch.float32)
        if key == "fp32":
            m = self.master[og][lo:lo + b - a]
            return _split_join(g.shard[a:b].to(self.device), m) if self.split_master else m
        st = self.optimizer.state.get(self.fp32_flat[og], {})
        t = st.get(key)
        return None if t is None else t[lo:lo + b - a]

    def _run_write(self, g, run, key, a, values, also_shard=False):
        s, e, og, moff, on_host = run
        lo = moff + a - s
        n = values.numel()
        values = values.reshape(-1).to(torch.float32)
        if key == "fp32" and self.split_master:
            hi, res = _split_cut(values.to(self.device))
            g.shard[a:a + n].copy_(hi)  # the weight IS the upper half of the master
            if on_host:
                self.off.write_state(og, "residual", lo, res)
            else:
                self.master[og][lo:lo + n].copy_(res)
            return
        if on_host:
            self.off.write_state(og, key, lo, values)
        elif key == "fp32":
            self.master[og][lo:lo + n].copy_(values)
        else:
            self._moments(og)[key][lo:lo + n].copy_(values)
        if key == "fp32" and also_shard:
            g.shard[a:a + n].copy_(values)

    def _frozen_full(self, g):
        """Gathered flat buffer of a frozen group (its 16-bit weights are the only state it has)."""
        shard = g.shard if g.shard.device == self.device else g.shard.to(self.device)
        if not g.partition:
            return shard
        full = torch.empty(g.padded, dtype=shard.dtype, device=self.device)
        dist.all_gather_into_tensor(full, shard.contiguous(), group=g.dp_group)
        return full

    @torch.no_grad()
    def _gather_param(self, p, key):
        self.join_offload()
        g, i = self.param_group[id(p)]
        if g.frozen:
            if key != "fp32":
                return None
            return self._frozen_full(g)[g.offsets[i]:g.offsets[i] + g.numels[i]].view(p.ds_shape).float()
        seg32 = torch.zeros(g.seg, dtype=torch.float32, device=self.device)
        for run in g.runs:
            src = self._run_read(g, run, key, run[0], run[1])
            if src is not None:
                seg32[run[0]:run[1]].copy_(src)
        if g.partition:
            full = torch.empty(g.padded, dtype=torch.float32, device=self.device)
            dist.all_gather_into_tensor(full, seg32, group=g.dp_group)
        else:
            full = seg32
        return full[g.offsets[i]:g.offsets[i] + g.numels[i]].view(p.ds_shape).clone()

    @torch.no_grad()
    def _scatter_param(self, p, value, key, also_shard=False):
        self.join_offload()
        g, i = self.param_group[id(p)]
        flat = value.reshape(-1).to(torch.float32)
        a = g.offsets[i]
        if g.frozen:
            if key == "fp32":
                lo, hi = max(g.seg_lo, a), min(g.seg_lo + g.seg, a + g.numels[i])
                if lo < hi:
                    g.shard[lo - g.seg_lo:hi - g.seg_lo].copy_(flat[lo - a:hi - a])
            return
        for run in g.runs:
            lo, hi = g.seg_lo + run[0], g.seg_lo + run[1]
            x0, x1 = max(lo, a), min(hi, a + g.numels[i])
            if x0 < x1:
                self._run_write(g, run, key, x0 - g.seg_lo, flat[x0 - a:x1 - a], also_shard=also_shard)

    def _local_fragment(self, p, key):
        """Elements of `p` owned by this rank's partition (flat fp32), or None."""
        self.join_offload()
        g, i = self.param_group[id(p)]
        a, n = g.offsets[i], g.numels[i]
        if g.frozen:
            lo, hi = max(g.seg_lo, a), min(g.seg_lo + g.seg, a + n)
            if key != "fp32" or lo >= hi:
                return None
            return g.shard[lo - g.seg_lo:hi - g.seg_lo].to(self.device, torch.float32)
        parts = []
        for run in g.runs:
            lo, hi = g.seg_lo + run[0], g.seg_lo + run[1]
            x0, x1 = max(lo, a), min(hi, a + n)
            if x0 < x1:
                src = self._run_read(g, run, key, x0 - g.seg_lo, x1 - g.seg_lo)
                if src is not None:
                    parts.append(src)
        return torch.cat(parts).clone() if parts else None

    def get_full_fp32_param(self, p):
        """Gather the fp32 master value of one parameter (reference `safe_get_full_fp32_param`)."""
        return self._gather_param(p, "fp32")

    def _ensure_state(self, key=None):
        """Materialise (zero) Adam moments for every optimizer group so they can be written into."""
        for og in range(len(self.fp32_flat)):
            self._moments(og)
            if self.off is not None:
                self.off._ensure_moments(og)

    def set_step(self, step):
        for og in range(len(self.fp32_flat)):
            st = self.optimizer.state[self.fp32_flat[og]]
            if "step" in st:
                st["step"] = int(step)
            if self.off is not None:
                self.off.step_count[og] = int(step)

    def get_full_optimizer_state(self, p, key):
        return self._gather_param(p, key)

    @torch.no_grad()
    def set_full_optimizer_state(self, p, value, key):
        self._scatter_param(p, value, key)

    def get_local_fp32_param(self, p):
        return self._local_fragment(p, "fp32")

    @torch.no_grad()
    def set_local_fragment(self, p, value, key):
        """Write back what `_local_fragment(p, key)` returned (same flat element order): this rank's part only, no
        collective."""
        self.join_offload()
        g, i = self.param_group[id(p)]
        a, n = g.offsets[i], g.numels[i]
        flat = value.reshape(-1).to(torch.float32)
        if g.frozen:
            lo, hi = max(g.seg_lo, a), min(g.seg_lo + g.seg, a + n)
            if key == "fp32" and lo < hi:
                g.shard[lo - g.seg_lo:hi - g.seg_lo].copy_(flat[:hi - lo])
            return
        off = 0
        for run in g.runs:
            lo, hi = g.seg_lo + run[0], g.seg_lo + run[1]
            x0, x1 = max(lo, a), min(hi, a + n)
            if x0 < x1:
                self._run_write(g, run, key, x0 - g.seg_lo, flat[off:off + x1 - x0], also_shard=key == "fp32")
                off += x1 - x0
        if off != flat.numel():
            raise ValueError(f"local fragment has {off} elements on this rank, got {flat.numel()}")

    def set_local_fp32_param(self, p, value):
        self.set_local_fragment(p, value, "fp32")

    def set_local_optimizer_state(self, p, value, key):
        self.set_local_fragment(p, value, key)

    def get_local_optimizer_state(self, p, key):
        return self._local_fragment(p, key)

    @torch.no_grad()
    def set_full_fp32_param(self, p, value):
        g, i = self.param_group[id(p)]
        self._scatter_param(p, value, "fp32", also_shard=True)
        if g.persistent and g.partition:
            dist.all_gather_into_tensor(g.full, g.shard, group=g.dp_group)

    @torch.no_grad()
    def get_full_grad(self, p):
        """Averaged fp32 gradient of one param (valid between backward at the boundary and step)."""
        g, i = self.param_group[id(p)]
        if g.frozen:
            return None
        seg32 = torch.zeros(g.seg, dtype=torch.float32, device=self.device)
        if g.mode == self.LOCAL:
            if p.grad is not None:
                seg32[g.offsets[i]:g.offsets[i] + g.numels[i]].copy_(p.grad.reshape(-1)).mul_(1.0 / self._div(g))
        elif g._acc_valid:
            for (s, e, og, moff, on_host) in g.runs:
                if not on_host:
                    seg32[s:e].copy_(self.grad_acc[og][moff:moff + e - s])
        elif g.red_out is not None:
            seg32.copy_(g.red_out).mul_(self._alpha(g))
        for piece in g.pieces:  # offloaded runs: the gradient sits in its host staging slot / accumulator
            if piece.covered and self.off is not None:
                self.off._drain()
                if self.off.cuda:
                    self.off.d2h.synchronize()
                src = self.off._grad_src(piece, piece.moff, piece.moff + piece.n)
                seg32[piece.s:piece.s + piece.n].copy_(src.to(self.device, torch.float32)).mul_(piece.alpha)
        seg32.mul_(self._unscale_factor())
        if g.partition:
            full = torch.empty(g.padded, dtype=torch.float32, device=self.device)
            dist.all_gather_into_tensor(full, seg32, group=g.dp_group)
        else:
            full = seg32
        return full[g.offsets[i]:g.offsets[i] + g.numels[i]].view(p.ds_shape).clone()

    def layout(self):
        """Describe the flat layout (for checkpoints / zero_to_fp32 / elastic reload): per group the param names,
        shapes, offsets, segment geometry, the runs (segment slice -> optimizer-group master offset), and for MoE
        expert groups the GLOBAL checkpoint name of every expert parameter (expert-parallel ranks hold different
        experts under the same local names)."""
        from ...checkpoint.zero_checkpoint import global_param_names
        names = {id(p): n for n, p in self.module.named_parameters()}
        gnames = global_param_names(self.module)
        out = []
        for g in self.groups:
            og0 = self.param_to_og[id(g.params[0])]
            moe = self.optimizer.param_groups[og0].get("moe", False)
            entry = dict(seg=g.seg, dp=g.dp, persistent=g.persistent, partition=bool(g.partition),
                         seg_lo=int(g.seg_lo), padded=int(g.padded), rank=int(g.rank),
                         params=[(names.get(id(p), f"param_{id(p)}"), list(p.ds_shape), g.offsets[i], g.numels[i])
                                 for i, p in enumerate(g.params)],
                         runs=[(s, e, og, moff, on_host) for (s, e, og, moff, on_host) in g.runs])
            if moe:
                entry["moe_group"] = self.optimizer.param_groups[og0].get("name")
                entry["global_names"] = {n: gnames.get(n, n) for (n, _, _, _) in entry["params"]}
            out.append(entry)
        return out

    # ================================================================================ checkpoint state
    def _device_master_fp32(self, og):
        """fp32 master of og's device-resident elements (joined from weight + residual with split masters)."""
        if not self.split_master:
            return self.master[og].detach().cpu()
        out = torch.zeros(self.master[og].numel(), dtype=torch.float32)
        for g in self.groups:
            for run in g.runs:
                if run[2] == og and not run[4]:
                    out[run[3]:run[3] + run[1] - run[0]].copy_(self._run_read(g, run, "fp32", run[0], run[1]))
        return out

    def _host_master_fp32(self, og):
        if self.off is None or self.off.n[og] == 0:
            return None
        if not self.split_master:
            return self.off.read_state(og, "fp32", 0, self.off.n[og]).clone()
        out = torch.zeros(self.off.n[og], dtype=torch.float32)
        for p in self.off.pieces[og]:
            run = (p.s, p.s + p.n, og, p.moff, True)
            out[p.moff:p.moff + p.n].copy_(self._run_read(p.group, run, "fp32", p.s, p.s + p.n))
        return out

    def state_dict(self, exclude_frozen_parameters=False):
        self.join_offload()
        sd = OrderedDict()
        sd[CK.ZERO_STAGE] = self.stage
        sd[CK.LOSS_SCALER] = self.loss_scaler.state_dict()
        sd["dynamic_loss_scale"] = self.dynamic_loss_scale
        sd["overflow"] = self.overflow
        sd[CK.CLIP_GRAD] = self.clip_grad
        sd[CK.PARTITION_COUNT] = self.partition_count()
        sd[CK.BASE_OPTIMIZER_STATE] = self.optimizer.state_dict()
        sd[CK.SINGLE_PARTITION_OF_FP32_GROUPS] = [self._device_master_fp32(og) for og in range(self.num_og)]
        sd["fp32_host_partitions"] = [self._host_master_fp32(og) for og in range(self.num_og)]
        sd["host_optimizer_states"] = {}
        if self.off is not None:
            for og in range(self.num_og):
                if self.off.n[og] and (self.off.step_count[og] or self.off.m[og] is not None):
                    self.off._ensure_moments(og)
                    n = self.off.n[og]
                    sd["host_optimizer_states"][og] = [self.off.read_state(og, "exp_avg", 0, n).clone(),
                                                       self.off.read_state(og, "exp_avg_sq", 0, n).clone(),
                                                       self.off.step_count[og]]
        sd[CK.FLAT_LAYOUT] = self.layout()
        if self.frozen_groups and not exclude_frozen_parameters:
            sd["frozen_layout"] = self.frozen_layout()
            sd["frozen_shards"] = [g.shard.detach().to("cpu").clone() for g in self.frozen_groups]
        sd[CK.DS_VERSION] = _version()
        return sd

    def frozen_layout(self):
        """Per frozen group: segment geometry and (name, shape, offset, numel) of its parameters, so any reader can
        cut every parameter out of the ranks' shards (reference: `frozen_param_fragments`, `engine.py:3432-3460`)."""
        names = {id(p): n for n, p in self.module.named_parameters()}
        return [dict(seg=g.seg, dp=g.dp, seg_lo=int(g.seg_lo), padded=int(g.padded), rank=int(g.rank),
                     partition=bool(g.partition),
                     params=[(names.get(id(p), f"param_{id(p)}"), list(p.ds_shape), g.offsets[i], g.numels[i])
                             for i, p in enumerate(g.params)]) for g in self.frozen_groups]

    @torch.no_grad()
    def load_frozen_shards(self, sd):
        """Positional restore of the frozen shards when the saved geometry is this rank's; returns False otherwise
        (the caller then rebuilds them from every rank's file, `checkpoint/zero_checkpoint.restore_frozen`)."""
        if not self.frozen_groups:
            return True
        if sd.get("frozen_layout") != self.frozen_layout():
            return False
        for g, t in zip(self.frozen_groups, sd["frozen_shards"]):
            g.shard.copy_(t)
        return True

    @torch.no_grad()
    def load_state_dict(self, sd, load_optimizer_states=True, load_from_fp32_weights=True):
        self.join_offload()
        if load_optimizer_states:
            base = sd[CK.BASE_OPTIMIZER_STATE]
            # our flat params are the optimizer params; restore states tensor-by-tensor onto device
            saved_groups = base["param_groups"]
            for og, group in enumerate(self.optimizer.param_groups):
                for k, v in saved_groups[og].items():
                    if k != "params":
                        group[k] = v
            for og, fp in enumerate(self.fp32_flat):
                key = base["param_groups"][og]["params"][0]
                st = base["state"].get(key, {})
                self.optimizer.state[fp] = {
                    k: (v.to(self.device) if torch.is_tensor(v) and v.dim() > 0 else v)
                    for k, v in st.items()
                }
            for og, s in sd.get("host_optimizer_states", {}).items():
                og = int(og)
                if self.off is not None and self.off.n[og]:
                    self.off.write_state(og, "exp_avg", 0, s[0])
                    self.off.write_state(og, "exp_avg_sq", 0, s[1])
                    self.off.step_count[og] = int(s[2])
        if CK.LOSS_SCALER in sd:
            ls = sd[CK.LOSS_SCALER]
            if isinstance(ls, dict):
                self.loss_scaler.load_state_dict(ls)
            else:
                self.loss_scaler = ls
        self.dynamic_loss_scale = sd.get("dynamic_loss_scale", self.dynamic_loss_scale)
        self.overflow = sd.get("overflow", False)
        if load_from_fp32_weights:
            dev = sd[CK.SINGLE_PARTITION_OF_FP32_GROUPS]
            host = sd.get("fp32_host_partitions", [])
            for g in self.groups:
                for run in g.runs:
                    (s, e, og, moff, on_host) = run
                    src = (host if on_host else dev)[og][moff:moff + e - s]
                    self._run_write(g, run, "fp32", s, src.to(self.device), also_shard=True)
            self._post_step_gather()
        if "frozen_shards" in sd:
            self.load_frozen_shards(sd)

    def refresh_from_module(self):
        """Re-read master weights from the (possibly externally modified) bf16 shards."""
        self.join_offload()
        for g in self.groups:
            for run in g.runs:
                self._run_write(g, run, "fp32", run[0], g.shard[run[0]:run[1]].float().to(self.device))


def _split_join(hi, lo):
    from .offload import split_join
    return split_join(hi.contiguous(), lo)


def _split_cut(f32):
    from .offload import split_cut
    return split_cut(f32)


class _nullctx:

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _host_zeros(n, dtype, pin):
    """Zeroed host buffer; pinned ones are allocated at their exact size (torch's pinned pool rounds every request
    up to a power of two, which would waste up to half of a Twin-Flow partition's host memory)."""
    if pin:
        from ...ops.native import hip_ops
        t = hip_ops().alloc_pinned(int(n), dtype)
        t.zero_()
        return t
    return torch.zeros(int(n), dtype=dtype)


def _devname(d):
    return str(getattr(d, "value", d))


def _version():
    from ... import __version__
    return __version__


# Reference-named entry points -------------------------------------------------------------------------------
class DeepSpeedZeroOptimizer(FlatZeroOptimizer):
    """ZeRO stage 1/2 (reference `runtime/zero/stage_1_and_2.py:96`)."""


class DeepSpeedZeroOptimizer_Stage3(FlatZeroOptimizer):
    """ZeRO stage 3 (reference `runtime/zero/stage3.py:73`)."""


class BF16_Optimizer(FlatZeroOptimizer):
    """bf16 params + fp32 master without ZeRO partitioning (reference `runtime/bf16_optimizer.py:30`)."""


class FP16_Optimizer(FlatZeroOptimizer):
    """fp16 params + fp32 master + dynamic loss scale (reference `runtime/fp16/fused_optimizer.py:31`)."""


# ------------------------------------------------------------------------------------------------ memory estimators
def model_to_params(model):
    """(total parameters, parameters of the largest top-level-leaf layer) of a model."""
    total = sum(p.numel() for p in model.parameters())
    largest = max((sum(p.numel() for p in m.parameters(recurse=False)) for m in model.modules()), default=0)
    return total, largest


def estimate_zero2_model_states_mem_needs(total_params, num_gpus_per_node=1, num_nodes=1, cpu_offload=True,
                                          additional_buffer_factor=1.5):
    """(host bytes per node, device bytes per GPU) for the model states under ZeRO-2 (reference
    `stage_1_and_2.py:2396-2420`): 16-bit weights + gradients replicated (4 B / param); the fp32 master, the two
    Adam moments and the fp32 gradient (16 B / param) split over all GPUs, or kept on the host."""
    total_gpus = num_nodes * num_gpus_per_node
    if cpu_offload:
        gpu_mem = 2 * total_params
        cpu_mem = total_params * max(4 * total_gpus, 16) * additional_buffer_factor
    else:
        gpu_mem = 4 * total_params + int(16 * total_params / total_gpus)
        cpu_mem = total_params * 4 * num_gpus_per_node * additional_buffer_factor
    return int(cpu_mem), int(gpu_mem)


def estimate_zero3_model_states_mem_needs(total_params, largest_layer_params, num_gpus_per_node=1, num_nodes=1,
                                          cpu_offload=True, cpu_offload_params=True, zero_init=True,
                                          additional_buffer_factor=1.5):
    """(host bytes per node, device bytes per GPU, bytes of the largest layer) under ZeRO-3 (reference
    `stage3.py:2613-2660`): everything is split over the GPUs (18 B / param) unless offloaded; the largest layer
    must be resident gathered (4 B / param: weights + gradients)."""
    total_gpus = num_nodes * num_gpus_per_node
    gpus_factor = 1 / num_nodes
    largest_layer_memory = 4 * largest_layer_params
    if cpu_offload:
        if cpu_offload_params:
            gpu_mem = largest_layer_memory
            per = 18
        else:
            gpu_mem = largest_layer_memory + int(2 * total_params / total_gpus)
            per = 16
        cpu_mem = total_params * per * gpus_factor * additional_buffer_factor if zero_init else \
            total_params * max(4 * num_gpus_per_node, per * gpus_factor) * additional_buffer_factor
    else:
        gpu_mem = largest_layer_memory + int(18 * total_params / total_gpus)
        cpu_mem = (largest_layer_params if zero_init else total_params) * 4 * num_gpus_per_node * \
            additional_buffer_factor
    return int(cpu_mem), int(gpu_mem), largest_layer_memory


def _gb(n):
    return f"{n / 2**30:7.2f}GB"


def estimate_zero2_model_states_mem_needs_all_cold(total_params, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    """Print the ZeRO-2 table (offload on / off) for a parameter count; returns the rows."""
    rows = []
    print(f"Estimated memory needed for params, optim states and gradients for a:\nHW: Setup with {num_nodes} "
          f"node{'s' if num_nodes > 1 else ''}, {num_gpus_per_node} GPU{'s' if num_gpus_per_node > 1 else ''} per "
          f"node.\nSW: Model with {int(total_params / 1e6)}M total params.\n  per CPU  |  per GPU |   Options")
    for off in (True, False):
        cpu, gpu = estimate_zero2_model_states_mem_needs(total_params, num_gpus_per_node, num_nodes, off,
                                                         additional_buffer_factor)
        rows.append({"offload_optimizer": off, "cpu": cpu, "gpu": gpu})
        print(f" {_gb(cpu)} | {_gb(gpu)} | offload_optimizer={'cpu' if off else 'none'}")
    return rows


def estimate_zero2_model_states_mem_needs_all_live(model, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    return estimate_zero2_model_states_mem_needs_all_cold(model_to_params(model)[0], num_gpus_per_node, num_nodes,
                                                          additional_buffer_factor)


def estimate_zero3_model_states_mem_needs_all_cold(total_params, largest_layer_params, num_gpus_per_node=1,
                                                   num_nodes=1, additional_buffer_factor=1.5):
    rows = []
    print(f"Estimated memory needed for params, optim states and gradients for a:\nHW: Setup with {num_nodes} "
          f"node{'s' if num_nodes > 1 else ''}, {num_gpus_per_node} GPU{'s' if num_gpus_per_node > 1 else ''} per "
          f"node.\nSW: Model with {int(total_params / 1e6)}M total params, {int(largest_layer_params / 1e6)}M "
          f"largest layer params.\n  per CPU  |  per GPU |   Options")
    for off_p, off_o in ((True, True), (False, True), (False, False)):
        for zi in (True, False):
            cpu, gpu, _ = estimate_zero3_model_states_mem_needs(total_params, largest_layer_params,
                                                                num_gpus_per_node, num_nodes, off_o, off_p, zi,
                                                                additional_buffer_factor)
            rows.append({"offload_param": off_p, "offload_optimizer": off_o, "zero_init": zi, "cpu": cpu,
                         "gpu": gpu})
            print(f" {_gb(cpu)} | {_gb(gpu)} | offload_param={'cpu' if off_p else 'none'}, offload_optimizer="
                  f"{'cpu' if off_o else 'none'}, zero_init={int(zi)}")
    return rows


def estimate_zero3_model_states_mem_needs_all_live(model, num_gpus_per_node=1, num_nodes=1,
                                                   additional_buffer_factor=1.5):
    total, largest = model_to_params(model)
    return estimate_zero3_model_states_mem_needs_all_cold(total, largest, num_gpus_per_node, num_nodes,
                                                          additional_buffer_factor)

