"""Slicing of fused QKV weights for tensor parallelism (reference `module_inject/fusedqkv_utils.py`).

A fused projection stores q, k and v along its output features in one of three orders; a rank's shard must hold whole
heads of each of the three, so the slice depends on the order:
  * "blocks"      [q | k | v]                      (GPT-2 c_attn, Phi Wqkv / qkv_proj): slice each third, re-join;
  * "interleaved" [head0: q k v | head1: q k v ..] (BLOOM / GPT-NeoX query_key_value): a contiguous row range;
  * "grouped"     [group: q..q k v | ...]          (Falcon multi-query): a contiguous range of groups.
"""
import torch

from .tp_shard import get_shard_size, get_shard_size_list

_ORDER_BY_NAME = {
    "c_attn": "blocks", "qkv_proj": "blocks", "Wqkv": "blocks", "W_pack": "blocks", "qkv": "blocks",
    "query_key_value": "interleaved",
}
_ORDER_BY_MODEL = {
    "CodeGenBlock": "codegen", "BloomBlock": "interleaved", "GPTNeoXLayer": "interleaved", "FalconDecoderLayer":
    "interleaved", "GLMBlock": "glm", "MPTBlock": "blocks", "BaichuanLayer": "blocks", "QWenBlock": "blocks",
    "PhiDecoderLayer": "blocks",
}


def require_tp_fused_qkvw(name, mp_size):
    """Does the parameter / module called `name` hold a fused QKV weight that needs order-aware slicing?"""
    if mp_size <= 1:
        return False
    leaf = name.replace(".weight", "").replace(".bias", "").split(".")[-1]
    return leaf in _ORDER_BY_NAME


def _split_blocks(src, mp_size, rank, parts=3):
    chunks = src.chunk(parts, dim=0)
    sizes = get_shard_size_list(chunks[0].shape[0], mp_size)
    lo = sum(sizes[:rank])
    return torch.cat([c[lo:lo + sizes[rank]] for c in chunks], dim=0)


def _split_rows(src, mp_size, rank):
    sizes = get_shard_size_list(src.shape[0], mp_size)
    lo = sum(sizes[:rank])
    return src[lo:lo + sizes[rank]]


def split_by_qkvlist_and_refuse(qkv_list, split_size, split_dim=0, cat_dim=0):
    """Split each of q, k, v into pieces of `split_size` along `split_dim` and re-fuse piece i of all three:
    returns one fused tensor per piece."""
    pieces = [torch.split(t, split_size, dim=split_dim) for t in qkv_list]
    return [torch.cat([p[i] for p in pieces], dim=cat_dim) for i in range(len(pieces[0]))]


def prepare_tp_fused_qkvw(module, src, mp_size, gpu_index):
    """This rank's rows of a fused QKV weight or bias `src` ([3 * width (, in)]): `module` (the block or the linear,
    or its class name) selects the storage order."""
    if src is None:
        return None
    name = module if isinstance(module, str) else type(module).__name__
    order = _ORDER_BY_MODEL.get(name) or _ORDER_BY_NAME.get(name.split(".")[-1], "blocks")
    if order == "interleaved":
        return _split_rows(src, mp_size, gpu_index)
    if order == "codegen":
        # CodeGen stores 4 model-parallel blocks of [q | v | k]: regroup to q, k, v, slice, and keep the block order
        mp_blocks = 4
        blocks = src.reshape(mp_blocks, 3, src.shape[0] // (3 * mp_blocks), *src.shape[1:])
        per = mp_blocks // mp_size if mp_blocks % mp_size == 0 else None
        if per is None:
            raise ValueError("CodeGen fused QKV is stored in 4 blocks: the tensor-parallel degree must divide 4")
        return blocks[gpu_index * per:(gpu_index + 1) * per].reshape(-1, *src.shape[1:])
    if order == "glm":
        # ChatGLM: [q (all heads) | k (kv heads) | v (kv heads)] with fewer kv heads
        from .tp_shard import get_num_kv_heads
        kv = get_num_kv_heads()
        if kv is None:
            return _split_blocks(src, mp_size, gpu_index)
        total = src.shape[0]
        # q takes the rest
        head_rows = None
        for hr in (256, 128, 96, 80, 64, 32):
            if (total - 2 * kv * hr) > 0 and (total - 2 * kv * hr) % hr == 0:
                head_rows = hr
                break
        if head_rows is None:
            return _split_blocks(src, mp_size, gpu_index)
        q, k, v = src.split([total - 2 * kv * head_rows, kv * head_rows, kv * head_rows], dim=0)
        return torch.cat([_split_rows(t, mp_size, gpu_index) for t in (q, k, v)], dim=0)
    return _split_blocks(src, mp_size, gpu_index)


__all__ = ["require_tp_fused_qkvw", "prepare_tp_fused_qkvw", "split_by_qkvlist_and_refuse", "get_shard_size"]
