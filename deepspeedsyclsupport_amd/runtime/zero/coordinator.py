"""ZeRO-3 parameter fetch / release / prefetch (reference `runtime/zero/partitioned_param_coordinator.py:58-526`
and the module hooks of `parameter_offload.py:342-540`).

Per fetch group (one module's params in one flat buffer):
  forward pre-hook  -> fetch (wait for an in-flight prefetch or gather now), then prefetch ahead along the trace
  forward hook      -> release (unless we are inside a backward recompute)
  backward pre-hook -> fetch again (params for the module's backward)
  all grads ready   -> release (from the optimizer's grad hook)
The trace of group fetches is recorded on the first step and replayed: at trace position i the coordinator issues
`all_gather_into_tensor` on the dedicated `ag_stream` for the next groups up to `prefetch_bucket_size` elements,
so xGMI transfers run under the current layer's GEMMs. A divergent fetch order invalidates the trace (re-record).

Reuse distance (reference `stage3_max_reuse_distance`, `partitioned_param_coordinator.py:389-416`): after a
module's forward, a group whose next fetch in the trace comes within `max_reuse_distance` gathered elements stays
gathered (within `max_live_parameters`). Sized for 288 GB of HBM — a 7B model's full bf16 weights are 13.4 GB — the
last layers' (or, with a large budget, every layer's) forward gather is reused by the backward instead of being
re-gathered over xGMI: one all-gather per parameter per step instead of two.
"""
import torch

from ... import comm as dist
from ...utils.logging import logger
from .flat_optimizer import ZeroParamStatus
from .linear import install_zero3_linear
from ...utils.nvtx import instrument_w_nvtx

RECORD, COMPLETE, INVALID = 0, 1, 2


class ParamCoordinator:

    def __init__(self, opt, prefetch_bucket_size=int(5e7), max_live_parameters=int(1e9),
                 max_reuse_distance=int(1e9)):
        self.opt = opt
        self.prefetch_bucket_size = int(prefetch_bucket_size)
        self.max_live = int(max_live_parameters)
        self.max_reuse = int(max_reuse_distance)
        self._reuse_dist = []  # per trace position: gathered elements until the same group's next fetch (or None)
        from .partitioned_param_profiler import PartitionedParameterProfiler
        self.profiler = PartitionedParameterProfiler(getattr(opt, "timers", None))
        self.trace = []
        self.mode = RECORD
        self.pos = 0
        self.in_backward = False
        self.ag_stream = opt.ag_stream
        self.acc = opt.acc
        self._hooks = []
        self.live_numel = 0
        # ZeRO++ (qwZ quantized weight gather, hpZ intra-node secondary partitions)
        zc = opt.zc
        self.qwz = bool(zc is not None and zc.zero_quantized_weights)
        # reference `zero_quantized_nontrainable_weights`: frozen weights travel as int8 blocks even when the trained
        # ones are gathered in 16 bits
        self.qnt = bool(zc is not None and zc.zero_quantized_nontrainable_weights)
        self.hpz = None
        if zc is not None and zc.zero_hpz_partition_size > 1 and opt.dp > zc.zero_hpz_partition_size:
            from ...parallel import groups
            from .zeropp import HpzState
            if not groups._zero_param_parallel_is_initialized():
                groups._create_zero_param_parallel_group(zc.zero_hpz_partition_size)
            self.hpz = HpzState(groups._get_zero_param_intra_parallel_group())
        install_zero3_linear(opt.module)
        self._deferred = []  # frozen groups whose release waits for the end of backward
        for g in opt.all_groups:
            if g.persistent or g.module is None:
                continue
            m = g.module
            first = "_ds_fetch_groups" not in m.__dict__
            m.__dict__.setdefault("_ds_fetch_groups", []).append(g)  # (trained and frozen params of one module)
            if first:
                self._hooks.append(m.register_forward_pre_hook(self._pre_fwd))
                self._hooks.append(m.register_forward_hook(self._post_fwd))
                self._hooks.append(m.register_full_backward_pre_hook(self._pre_bwd))
            if g.frozen and not m.__dict__.get("_ds_frozen_hooked"):
                # trained groups are released when their last gradient arrives; frozen ones produce none, so the
                # module's backward hook (input gradients computed) releases them
                m.__dict__["_ds_frozen_hooked"] = True
                self._hooks.append(m.register_full_backward_hook(self._post_bwd))
        for m in opt.module.modules():
            if m.__dict__.get("_ds_external_params"):
                self.install_external(m)

    # ----------------------------------------------------------------------------------- external parameters
    def install_external(self, m):
        """Fetch hooks for the parameters `m` uses but does not own (`zero.register_external_parameter`). A group
        already gathered by its owner (nested use) is borrowed, not released, by `m`."""
        if m.__dict__.get("_ds_ext_hooked"):
            return
        m.__dict__["_ds_ext_hooked"] = True

        def groups_of(mod):
            seen, out = set(), []
            for p in mod.__dict__.get("_ds_external_params", []):
                g = getattr(p, "ds_group", None)
                if g is not None and not g.persistent and id(g) not in seen:
                    seen.add(id(g))
                    out.append(g)
            return out

        def pre(mod, inputs):
            mod.__dict__["_ds_ext_borrowed"] = {g.idx: g.status != ZeroParamStatus.NOT_AVAILABLE
                                                for g in groups_of(mod)}
            for g in groups_of(mod):
                self.fetch(g)

        def post(mod, inputs, outputs):
            if self.in_backward or torch._C._current_graph_task_id() != -1:
                return
            borrowed = mod.__dict__.get("_ds_ext_borrowed", {})
            for g in groups_of(mod):
                if not borrowed.get(g.idx, False):
                    self.release(g)

        def pre_bwd(mod, grad_output):
            for g in groups_of(mod):
                self.fetch(g)

        self._hooks.append(m.register_forward_pre_hook(pre))
        self._hooks.append(m.register_forward_hook(post))
        self._hooks.append(m.register_full_backward_pre_hook(pre_bwd))

    # ----------------------------------------------------------------------------------- hooks
    def _pre_fwd(self, m, inputs):
        for g in m._ds_fetch_groups:
            self.fetch(g)

    def _post_fwd(self, m, inputs, outputs):
        if self.in_backward or torch._C._current_graph_task_id() != -1:
            return  # activation-checkpoint recompute inside backward: keep params for the module's backward
        for g in m._ds_fetch_groups:
            if self._keep_for_reuse(g):
                self.profiler.count("reuse_hit", g.numel)
                continue
            self.release(g)

    def _keep_for_reuse(self, g):
        """Keep a just-used group gathered when the trace says it is fetched again soon enough."""
        if self.mode != COMPLETE or self.max_reuse <= 0 or g.persistent:
            return False
        p = getattr(g, "_ds_trace_pos", None)
        if p is None or p >= len(self._reuse_dist):
            return False
        d = self._reuse_dist[p]
        return d is not None and d <= self.max_reuse and self.live_numel <= self.max_live

    def _pre_bwd(self, m, grad_output):
        for g in m._ds_fetch_groups:
            self.fetch(g)

    def _post_bwd(self, m, grad_input, grad_output):
        frozen = [g for g in m._ds_fetch_groups if g.frozen]
        if all(gi is None for gi in grad_input):
            # no input needs a gradient: autograd fires this hook BEFORE the module's own backward work, so the
            # weights stay until the pass is over
            self._deferred.extend(frozen)
            return
        for g in frozen:
            self.release_after_backward(g)

    # ----------------------------------------------------------------------------------- core
    def _gather(self, g):
        """Fill g.full: hpZ intra-node re-gather in backward, qwZ int8 gather, or the plain bf16 all-gather.
        Offloaded shards (ZeRO-Infinity) are first streamed host->device on this same stream."""
        hpz = self.hpz if (self.hpz is not None and g.dp_group is self.opt.dp_group) else None
        if self.in_backward and hpz is not None and hpz.can_use(g):
            hpz.gather_from_secondary(g)
            return
        shard = g.shard
        if shard.device != g.full.device:
            if not g.partition:
                g.full[:g.seg].copy_(shard, non_blocking=shard.is_pinned())
                return
            staged = torch.empty(g.seg, dtype=shard.dtype, device=g.full.device)
            staged.copy_(shard, non_blocking=shard.is_pinned())
            shard = staged
        if not g.partition:
            g.full.copy_(shard)
        elif self.qwz or (self.qnt and g.frozen):
            from .zeropp import quantized_all_gather
            quantized_all_gather(g.full, shard, g.dp_group)
        elif getattr(self.opt, "mics_hier", None) is not None and g.dp_group is self.opt.mics_shard_group:
            from .zeropp import hierarchical_all_gather
            hierarchical_all_gather(g.full, shard, *self.opt.mics_hier)
        else:
            dist.all_gather_into_tensor(g.full, shard, group=g.dp_group)
        if hpz is not None and not self.in_backward:
            hpz.keep_secondary(g)

    @instrument_w_nvtx
    def _issue(self, g):
        opt = self.opt
        if g.status != ZeroParamStatus.NOT_AVAILABLE:
            return
        if opt.safe_mode and g.partition:
            from .utils import assert_ints_same_as_other_ranks
            assert_ints_same_as_other_ranks([g.idx, g.padded], g.dp_group, "parameter all-gather (group id, numel)")
        compute = self.acc.current_stream() if self.ag_stream is not None else None
        if self.ag_stream is not None:
            self.ag_stream.wait_stream(compute)
            with self.acc.stream(self.ag_stream):
                if opt.off is not None and g.pieces:
                    opt.off.wait_group(g)  # host-stepped weights of this shard must have landed (orders ag_stream)
                g.full = torch.empty(g.padded, dtype=opt.dtype, device=opt.device)
                self._gather(g)
                g.ag_event = self.acc.Event()
                g.ag_event.record(self.ag_stream)
        else:
            if opt.off is not None and g.pieces:
                opt.off.wait_group(g)
            g.full = torch.empty(g.padded, dtype=opt.dtype, device=opt.device)
            self._gather(g)
            g.ag_event = None
        g.status = ZeroParamStatus.INFLIGHT
        self.live_numel += g.padded
        self.profiler.count("all_gather", g.padded)

    def _wait(self, g):
        if g.status == ZeroParamStatus.INFLIGHT:
            if g.ag_event is not None:
                cur = self.acc.current_stream()
                cur.wait_event(g.ag_event)
                g.full.record_stream(cur)
            self.opt._point_params(g)
            g.status = ZeroParamStatus.AVAILABLE

    @instrument_w_nvtx
    def fetch(self, g):
        self.profiler.count("fetch", g.numel)
        self._trace(g)
        if g.status == ZeroParamStatus.NOT_AVAILABLE:
            self._issue(g)
        self._wait(g)
        self._prefetch()

    @instrument_w_nvtx
    def release(self, g):
        if g.persistent or g.status == ZeroParamStatus.NOT_AVAILABLE:
            return
        if g.status == ZeroParamStatus.INFLIGHT:
            self._wait(g)
        self.opt._release_params(g)
        g.full = None
        self.live_numel -= g.padded
        self.profiler.count("release", g.numel)

    def release_after_backward(self, g):
        self.release(g)
        if self.hpz is not None:
            self.hpz.drop(g)

    # ----------------------------------------------------------------------------------- trace / prefetch
    def _trace(self, g):
        if self.mode == RECORD:
            self.trace.append(g.idx)
            return
        if self.mode == COMPLETE:
            if self.pos < len(self.trace) and self.trace[self.pos] == g.idx:
                g._ds_trace_pos = self.pos
                self.pos += 1
            else:
                logger.debug("ZeRO-3 fetch order diverged from the recorded trace; re-recording")
                self.mode = INVALID

    def _prefetch(self):
        if self.mode != COMPLETE or self.prefetch_bucket_size <= 0:
            return
        budget = self.prefetch_bucket_size
        i = self.pos
        groups = self.opt.all_groups
        while i < len(self.trace) and budget > 0:
            g = groups[self.trace[i]]
            if g.status == ZeroParamStatus.NOT_AVAILABLE:
                if self.live_numel + g.padded > self.max_live:
                    break
                self._issue(g)
            budget -= g.numel
            i += 1

    def _reuse_distances(self):
        """For each trace position, the elements gathered between it and the next fetch of the same group."""
        groups = self.opt.all_groups
        prefix = [0]
        for gi in self.trace:
            prefix.append(prefix[-1] + groups[gi].numel)
        nxt, out = {}, [None] * len(self.trace)
        for p in range(len(self.trace) - 1, -1, -1):
            gi = self.trace[p]
            if gi in nxt:
                out[p] = prefix[nxt[gi]] - prefix[p + 1]
            nxt[gi] = p
        return out

    def begin_backward(self):
        self.in_backward = True

    def end_backward(self):
        self.in_backward = False
        for g in self._deferred:
            self.release_after_backward(g)
        self._deferred = []

    def reset_step(self):
        """End of an optimizer step: close the trace, release anything still gathered."""
        if self.mode == RECORD:
            if self.opt.safe_mode and self.trace:
                from .utils import assert_ints_same_as_other_ranks, trace_digest
                assert_ints_same_as_other_ranks(trace_digest(self.trace), self.opt.dp_group,
                                                "recorded ZeRO-3 fetch trace (length, digest)")
            self.mode = COMPLETE if self.trace else RECORD
            self._reuse_dist = self._reuse_distances()
        elif self.mode == INVALID:
            self.trace = []
            self.mode = RECORD
        self.pos = 0
        for g in self.opt.all_groups:
            if not g.persistent and g.status != ZeroParamStatus.NOT_AVAILABLE:
                self.release(g)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


class ZeRoTraceMode:
    """States of the module-order trace that drives prefetching (reference
    `partitioned_param_coordinator.py:38`): RECORD on the first step (and again whenever the order changes),
    COMPLETE once a step replayed the recorded order, INVALID when a mismatch disabled prefetching."""
    RECORD = 1
    COMPLETE = 2
    INVALID = 3


class InflightParamRegistry(dict):
    """param -> pending gather handle; a parameter may have at most one gather in flight."""

    def __setitem__(self, param, handle):
        if param in self:
            raise RuntimeError(f"{getattr(param, 'ds_id', id(param))} already in registry")
        super().__setitem__(param, handle)


def iter_params(module, recurse=False):
    return (p for _, p in module.named_parameters(recurse=recurse))


def get_all_parameters(sub_module, recurse=False):
    """Own parameters plus registered external ones (`register_external_parameter`)."""
    import itertools
    ext = getattr(sub_module, "_external_params", {})
    return itertools.chain(sub_module.named_parameters(recurse=recurse), ext.items())

