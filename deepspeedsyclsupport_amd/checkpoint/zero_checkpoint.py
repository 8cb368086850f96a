"""ZeRO checkpoint state at any topology: per-parameter reconstruction from rank shards, and restore into a live
flat-group optimizer at a (possibly different) data-parallel size.

Reference behaviour: elastic ZeRO-1/2 load (`runtime/zero/stage_1_and_2.py:2148-2237`
`_restore_from_elastic_fp32_weights` / `_restore_elastic_base_optimizer_state`: merge every rank's partition, re-slice
for the new partition), ZeRO-3 load (`stage3.py:2530`), consolidation (`utils/zero_to_fp32.py:468-533`) and the
engine's load path (`runtime/engine.py:2914-3020`).

Design: every source answers ONE question — "give me the full fp32 value (or Adam moment) of parameter `name`" —
and the restore walks the live optimizer's parameters, asks the source, and scatters each answer into this rank's
flat fp32 master / moment buffers and bf16 shard (`FlatZeroOptimizer._scatter_param`, no communication). Nothing
is ever gathered on a device, files are opened with `torch.load(mmap=True, weights_only=True)`, so a rank touches
only the pages that back the slices it needs and host memory stays at one parameter at a time.

Sources:
  * FlatLayoutSource      — this framework's `*_optim_states.pt` files (`ds_flat_layout` descriptor per rank), any
                            number of ranks, ZeRO-1/2/3, Twin-Flow host partitions, MoE expert groups (keyed by
                            GLOBAL expert id, so expert shards saved by different expert-parallel ranks never
                            collide).
  * ReferenceZero12Source — reference ZeRO-1/2 files: `single_partition_of_fp32_groups` per optimizer group,
                            `base_optimizer_state` (torch optimizer state of the flat partitions), flattened in
                            `param_shapes` order (`stage_1_and_2.py:2102-2146`, merged as `zero_to_fp32.py:233-290`).
  * ReferenceZero3Source  — reference ZeRO-3 files: `fp32_flat_groups` per sub-group, every parameter split into
                            `ceil(numel / world)` pieces per rank (`stage3.py:2382-2395`, `zero_to_fp32.py:330-390`).
No checkpoint written by the reference ships in `/root/reference`, so the reference-format readers are tested
against files synthesised from the reference's save code (parity with real files: unpinned).
"""
import glob
import math
import os
import re
from collections import OrderedDict

import torch

from . import constants as CK

_EXPERT_RE = re.compile(r"(.*\.deepspeed_experts\.)(\d+)(\..*)")


# ---------------------------------------------------------------------------------------------------- file access
_STUBS = {}


def _reference_pickle_stubs():
    """Allow-listed stand-ins for the few non-tensor objects the reference pickles into its checkpoints
    (`LossScaler` / `DynamicLossScaler` instances, `fragment_address` namedtuples, `ZeroStageEnum`), so that
    reference-format files load under `weights_only=True`. Nothing from the file is executed: the weights-only
    unpickler matches these inert classes by qualified name and only fills their `__dict__`. They are NOT installed
    in `sys.modules` (a fake `deepspeed` package would confuse library probes)."""
    if _STUBS:
        return list(_STUBS.values())
    specs = {
        "deepspeed.runtime.fp16.loss_scaler": ["LossScaler", "DynamicLossScaler", "LossScalerBase"],
        "deepspeed.runtime.zero.config": ["ZeroStageEnum"],
        "deepspeed.utils.tensor_fragment": ["fragment_address"],
    }
    for mod_name, classes in specs.items():
        for cname in classes:
            if cname == "fragment_address":
                from collections import namedtuple
                cls = namedtuple("fragment_address", ["numel", "start"])
            elif cname == "ZeroStageEnum":
                import enum
                cls = enum.IntEnum("ZeroStageEnum", [("disabled", 0), ("optimizer_states", 1), ("gradients", 2),
                                                     ("weights", 3)])
            else:
                cls = type(cname, (), {})
            cls.__module__ = mod_name
            cls.__qualname__ = cname
            _STUBS[f"{mod_name}.{cname}"] = cls
    return list(_STUBS.values())


def load_file(path, mmap=True):
    """torch.load that executes nothing from the file; memory-mapped when the format allows."""
    stubs = _reference_pickle_stubs()
    with torch.serialization.safe_globals(stubs):
        try:
            return torch.load(path, map_location="cpu", weights_only=True, mmap=mmap)
        except RuntimeError:
            if not mmap:
                raise
            return torch.load(path, map_location="cpu", weights_only=True)  # legacy (non-zip) format


def _rank_of(path):
    m = re.search(r"zero_pp_rank_(\d+)_mp_rank_(\d+)", os.path.basename(path))
    return (int(m.group(2)), int(m.group(1))) if m else (0, 0)


def optim_files(ckpt_dir, mp_rank=None):
    files = [f for f in glob.glob(os.path.join(ckpt_dir, f"*{CK.OPTIM_FILE_SUFFIX}")) if "zero_pp_rank_" in f]
    if mp_rank is not None:
        files = [f for f in files if _rank_of(f)[0] == mp_rank]
    return sorted(files, key=_rank_of)


def global_param_names(module):
    """{local parameter name: checkpoint name}. Expert parameters of a MoE layer are renamed with their GLOBAL expert
    id (expert-parallel rank * local experts + local id), the reference's expert-file convention
    (`runtime/engine.py:3151-3200`); every other name is unchanged."""
    out = {}
    moe_of = {}
    for mname, m in module.named_modules():
        if hasattr(m, "num_local_experts") and hasattr(m, "expert_group_name") and hasattr(m, "deepspeed_moe"):
            moe_of[mname] = m
    ep_rank_cache = {}
    for name, _ in module.named_parameters():
        out[name] = name
        mm = _EXPERT_RE.match(name)
        if not mm:
            continue
        owner = max((k for k in moe_of if name.startswith(k + ".") or k == ""), key=len, default=None)
        if owner is None:
            continue
        m = moe_of[owner]
        gname = m.expert_group_name
        if gname not in ep_rank_cache:
            try:
                from ..parallel import groups
                ep_rank_cache[gname] = groups._get_expert_parallel_rank(gname)
            except Exception:  # groups not initialised (single process)
                ep_rank_cache[gname] = 0
        gid = ep_rank_cache[gname] * m.num_local_experts + int(mm.group(2))
        out[name] = f"{mm.group(1)}{gid}{mm.group(3)}"
    return out


# ---------------------------------------------------------------------------------------------------- sources
class ShardSource:
    """Per-parameter full fp32 values / Adam moments from a set of rank shards."""
    keys = ("fp32", "exp_avg", "exp_avg_sq")

    def names(self):
        raise NotImplementedError

    def get(self, name, key="fp32"):
        raise NotImplementedError

    def step(self):
        return None

    def has_moments(self):
        return True


class FlatLayoutSource(ShardSource):
    """This framework's shards: every rank file carries `ds_flat_layout` (groups -> seg / seg_lo / runs / params)."""

    def __init__(self, files):
        if not files:
            raise FileNotFoundError("no ZeRO optimizer shards given")
        self.files = list(files)
        self.states = [load_file(f)[CK.OPTIMIZER_STATE_DICT] for f in self.files]
        # index: checkpoint name -> [(state idx, group entry, (shape, offset, numel))]
        self.index = OrderedDict()
        for si, st in enumerate(self.states):
            if CK.FLAT_LAYOUT not in st:
                raise ValueError(f"{self.files[si]} has no {CK.FLAT_LAYOUT}: not a flat-layout shard")
            for g in st[CK.FLAT_LAYOUT]:
                gnames = g.get("global_names") or {}
                for (name, shape, off, numel) in g["params"]:
                    key = gnames.get(name, name)
                    self.index.setdefault(key, []).append((si, g, (tuple(shape), off, numel)))
        # frozen parameters: name -> [(state idx, frozen group index, group entry, (shape, offset, numel))]
        self.frozen_index = OrderedDict()
        for si, st in enumerate(self.states):
            for gi, g in enumerate(st.get("frozen_layout") or []):
                for (name, shape, off, numel) in g["params"]:
                    self.frozen_index.setdefault(name, []).append((si, gi, g, (tuple(shape), off, numel)))

    def names(self):
        return list(self.index.keys())

    def frozen_names(self):
        return list(self.frozen_index.keys())

    def get_frozen(self, name):
        """Full value (saved dtype) of a frozen parameter cut out of the ranks' frozen shards, or None."""
        ent = self.frozen_index.get(name)
        if ent is None:
            return None
        shape, _, numel = ent[0][3]
        out, covered = None, torch.zeros(numel, dtype=torch.bool)
        for (si, gi, g, (_, off, _)) in ent:
            shard = self.states[si]["frozen_shards"][gi]
            lo = g["seg_lo"]
            a, b = max(lo, off), min(lo + g["seg"], off + numel)
            if a >= b:
                continue
            if out is None:
                out = torch.zeros(numel, dtype=shard.dtype)
            out[a - off:b - off] = shard[a - lo:b - lo]
            covered[a - off:b - off] = True
        if out is None or not bool(covered.all()):
            raise ValueError(f"checkpoint shards cover only {int(covered.sum())}/{numel} elements of frozen "
                             f"parameter '{name}' ({len(self.files)} files read)")
        return out.view(shape)

    def _fetch(self, st, key, og, on_host):
        if key == "fp32":
            if on_host:
                host = st.get("fp32_host_partitions") or []
                return host[og] if og < len(host) else None
            return st[CK.SINGLE_PARTITION_OF_FP32_GROUPS][og]
        idx = {"exp_avg": 0, "exp_avg_sq": 1}[key]
        if on_host:
            hs = (st.get("host_optimizer_states") or {})
            s = hs.get(og, hs.get(str(og)))
            return None if s is None else s[idx]
        base = st[CK.BASE_OPTIMIZER_STATE]
        pid = base["param_groups"][og]["params"][0]
        return base["state"].get(pid, {}).get(key)

    def get(self, name, key="fp32"):
        ent = self.index.get(name)
        if ent is None:
            return None
        shape, off, numel = ent[0][2]
        out = torch.zeros(numel, dtype=torch.float32)
        covered = torch.zeros(numel, dtype=torch.bool)
        seen_any = False
        for (si, g, (_, off_i, _)) in ent:
            st = self.states[si]
            lo = g["seg_lo"]
            for (s, e, og, moff, on_host) in g["runs"]:
                a, b = max(lo + s, off_i), min(lo + e, off_i + numel)
                if a >= b:
                    continue
                src = self._fetch(st, key, og, on_host)
                if src is None:
                    continue
                seen_any = True
                out[a - off_i:b - off_i] = src[moff + a - lo - s:moff + b - lo - s].float()
                covered[a - off_i:b - off_i] = True
        if not seen_any:
            return None
        if not bool(covered.all()):
            raise ValueError(f"checkpoint shards cover only {int(covered.sum())}/{numel} elements of '{name}': "
                             f"a data-parallel rank's file is missing ({len(self.files)} files read)")
        return out.view(shape)

    def step(self):
        for st in self.states:
            base = st.get(CK.BASE_OPTIMIZER_STATE) or {}
            for s in (base.get("state") or {}).values():
                if "step" in s:
                    v = s["step"]
                    return int(v.item() if torch.is_tensor(v) else v)
            for s in (st.get("host_optimizer_states") or {}).values():
                return int(s[2])
        return None

    def has_moments(self):
        return any((st.get(CK.BASE_OPTIMIZER_STATE) or {}).get("state") for st in self.states) or \
            any(st.get("host_optimizer_states") for st in self.states)


def _ref_param_shapes(model_file):
    ms = load_file(model_file)
    shapes = ms.get(CK.PARAM_SHAPES)
    if shapes is None:
        raise ValueError(f"{model_file} has no {CK.PARAM_SHAPES}: cannot place reference partitions")
    if isinstance(shapes, dict):
        shapes = [shapes]
    return [OrderedDict((k, tuple(v)) for k, v in d.items()) for d in shapes]


def _base_state_list(osd, n_groups):
    """Reference `base_optimizer_state`: a torch optimizer state_dict ({'state', 'param_groups'}) or, with
    elastic_checkpoint, a list of per-group state dicts."""
    base = osd.get(CK.BASE_OPTIMIZER_STATE, osd.get(CK.OPTIMIZER_STATE_DICT))
    if base is None:
        return [dict() for _ in range(n_groups)]
    if isinstance(base, (list, tuple)):
        return list(base)
    state = base.get("state", {})
    out = []
    for gi, g in enumerate(base.get("param_groups", [])):
        pid = g["params"][0] if g.get("params") else gi
        out.append(state.get(pid, {}))
    while len(out) < n_groups:
        out.append({})
    return out


class ReferenceZero12Source(ShardSource):
    """Reference ZeRO-1/2: per optimizer group the ranks' partitions concatenate to the group's flat tensor, whose
    parameters sit back to back in `param_shapes` order."""

    def __init__(self, files, model_file):
        self.files = files
        self.states = [load_file(f)[CK.OPTIMIZER_STATE_DICT] for f in files]
        self.shapes = _ref_param_shapes(model_file)
        self.flat = {}   # (key, group) -> merged flat tensor
        self.where = {}  # name -> (group, offset, shape)
        for gi, d in enumerate(self.shapes):
            off = 0
            for name, shape in d.items():
                self.where[name] = (gi, off, shape)
                off += int(math.prod(shape))

    def names(self):
        return list(self.where.keys())

    def _group_flat(self, key, gi):
        k = (key, gi)
        if k not in self.flat:
            parts = []
            for st in self.states:
                if key == "fp32":
                    parts.append(st[CK.SINGLE_PARTITION_OF_FP32_GROUPS][gi].float())
                else:
                    s = _base_state_list(st, len(st[CK.SINGLE_PARTITION_OF_FP32_GROUPS]))[gi]
                    if key not in s:
                        self.flat[k] = None
                        return None
                    n = st[CK.SINGLE_PARTITION_OF_FP32_GROUPS][gi].numel()
                    parts.append(s[key].reshape(-1)[:n].float())  # drop the last rank's alignment padding
            self.flat[k] = torch.cat(parts)
        return self.flat[k]

    def get(self, name, key="fp32"):
        if name not in self.where:
            return None
        gi, off, shape = self.where[name]
        flat = self._group_flat(key, gi)
        if flat is None:
            return None
        n = int(math.prod(shape))
        return flat[off:off + n].clone().view(shape)

    def step(self):
        for st in self.states:
            if CK.BASE_OPTIMIZER_STATE_STEP in st:
                return int(st[CK.BASE_OPTIMIZER_STATE_STEP])
            for s in _base_state_list(st, len(st[CK.SINGLE_PARTITION_OF_FP32_GROUPS])):
                if "step" in s:
                    v = s["step"]
                    return int(v.item() if torch.is_tensor(v) else v)
        return None


class ReferenceZero3Source(ShardSource):
    """Reference ZeRO-3: rank r holds piece r (ceil(numel / world) elements, zero padded) of every parameter, the
    pieces of all parameters concatenated over its sub-groups in `param_shapes` order."""

    def __init__(self, files, model_file):
        self.files = files
        self.states = [load_file(f)[CK.OPTIMIZER_STATE_DICT] for f in files]
        self.world = len(files)
        shapes = _ref_param_shapes(model_file)
        self.where = OrderedDict()
        off = 0
        for d in shapes:
            for name, shape in d.items():
                numel = int(math.prod(shape))
                pn = math.ceil(numel / self.world)
                self.where[name] = (off, pn, numel, shape)
                off += pn
        self.flat = {}

    def names(self):
        return list(self.where.keys())

    def _rank_flat(self, key, r):
        k = (key, r)
        if k not in self.flat:
            st = self.states[r]
            if key == "fp32":
                groups = st[CK.FP32_FLAT_GROUPS]
            else:
                inner = st.get(CK.OPTIMIZER_STATE_DICT) or {}
                state = inner.get("state", {})
                pg = inner.get("param_groups", [])
                ids = [i for g in pg for i in g.get("params", [])] or sorted(state.keys())
                groups = [state[i][key] for i in ids if i in state and key in state[i]]
                if not groups:
                    self.flat[k] = None
                    return None
            self.flat[k] = torch.cat([g.reshape(-1).float() for g in groups])
        return self.flat[k]

    def get(self, name, key="fp32"):
        if name not in self.where:
            return None
        off, pn, numel, shape = self.where[name]
        parts = []
        for r in range(self.world):
            f = self._rank_flat(key, r)
            if f is None:
                return None
            parts.append(f[off:off + pn])
        return torch.cat(parts)[:numel].clone().view(shape)

    def step(self):
        for st in self.states:
            inner = st.get(CK.OPTIMIZER_STATE_DICT) or {}
            for s in (inner.get("state") or {}).values():
                if "step" in s:
                    v = s["step"]
                    return int(v.item() if torch.is_tensor(v) else v)
        return None


def open_source(ckpt_dir, mp_rank=0):
    """Pick the reader for the shards in `ckpt_dir` (one tag directory)."""
    files = optim_files(ckpt_dir, mp_rank) or optim_files(ckpt_dir)
    if not files:
        raise FileNotFoundError(f"no zero_pp_rank_*{CK.OPTIM_FILE_SUFFIX} files in {ckpt_dir}")
    probe = load_file(files[0])[CK.OPTIMIZER_STATE_DICT]
    if CK.FLAT_LAYOUT in probe:
        return FlatLayoutSource(files)
    models = sorted(glob.glob(os.path.join(ckpt_dir, f"*{CK.MODEL_FILE_SUFFIX}")))
    models = [m for m in models if "expert_" not in os.path.basename(m)]
    if not models:
        raise FileNotFoundError(f"reference-format shards in {ckpt_dir} but no *{CK.MODEL_FILE_SUFFIX}")
    if CK.FP32_FLAT_GROUPS in probe:
        return ReferenceZero3Source(files, models[0])
    if CK.SINGLE_PARTITION_OF_FP32_GROUPS in probe:
        return ReferenceZero12Source(files, models[0])
    raise ValueError(f"unrecognised ZeRO shard format in {files[0]}")


# ---------------------------------------------------------------------------------------------------- restore
@torch.no_grad()
def restore_from_source(optimizer, module, source, load_optimizer_states=True, strict=True):
    """Scatter every parameter's fp32 master (and, when asked and present, Adam moments) from `source` into this
    rank's flat buffers; refresh bf16 shards and persistent full buffers. Returns the restored step (or None)."""
    gnames = global_param_names(module)
    names = {id(p): n for n, p in module.named_parameters()}
    want_moments = load_optimizer_states and source.has_moments()
    if want_moments:
        optimizer._ensure_state()
    missing = []
    for p in optimizer.opt_params:
        local = names.get(id(p))
        if local is None:
            continue
        key = gnames.get(local, local)
        v = source.get(key, "fp32")
        if v is None:
            missing.append(key)
            continue
        optimizer._scatter_param(p, v, "fp32", also_shard=True)
        if want_moments:
            for k in ("exp_avg", "exp_avg_sq"):
                m = source.get(key, k)
                if m is not None:
                    optimizer._scatter_param(p, m, k)
    if strict and missing:
        raise KeyError(f"checkpoint has no fp32 state for {len(missing)} parameter(s), e.g. {missing[:3]}")
    step = source.step() if want_moments else None
    if step is not None:
        optimizer.set_step(step)
    optimizer._post_step_gather()
    restore_frozen(optimizer, module, source)
    return step


@torch.no_grad()
def restore_frozen(optimizer, module, source):
    """Frozen (partitioned, optimizer-less) parameters saved under another partitioning: each one is cut out of the
    saving ranks' frozen shards and its local slice written into this rank's shard. Parameters the checkpoint does
    not hold (saved with exclude_frozen_parameters) keep their current values."""
    get = getattr(source, "get_frozen", None)
    if get is None:
        return 0
    owned = {id(p) for p in optimizer.opt_params}
    grouped = getattr(optimizer, "param_group", {})
    n = 0
    for name, p in module.named_parameters():
        if id(p) in owned:
            continue
        v = get(name)
        if v is None:
            continue
        if id(p) in grouped:
            optimizer._scatter_param(p, v, "fp32", also_shard=True)
        else:  # kept whole by this engine (one data-parallel rank, or below the persistence threshold)
            p.data.copy_(v.reshape(p.shape))
        n += 1
    return n


def layouts_match(saved, current):
    """Same flat layout (group structure, offsets, segments, runs) on this rank => positional load is exact."""
    if saved is None or len(saved) != len(current):
        return False
    for a, b in zip(saved, current):
        for k in ("seg", "dp", "partition", "seg_lo", "padded"):
            if a.get(k) != b.get(k):
                return False
        if [tuple(x[:1]) + (tuple(x[1]), ) + tuple(x[2:4]) for x in a["params"]] != \
                [tuple(x[:1]) + (tuple(x[1]), ) + tuple(x[2:4]) for x in b["params"]]:
            return False
        if [tuple(r) for r in a["runs"]] != [tuple(r) for r in b["runs"]]:
            return False
    return True


def __getattr__(name):
    # `ZeROCheckpoint` (folder inspection / contraction) lives with `DeepSpeedCheckpoint`; resolved lazily because
    # that module imports this one
    if name == "ZeROCheckpoint":
        from .deepspeed_checkpoint import ZeROCheckpoint
        return ZeROCheckpoint
    raise AttributeError(name)

