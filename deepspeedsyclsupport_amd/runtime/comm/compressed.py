"""Error-compensated 1-bit all-reduce (reference `runtime/comm/nccl.py:51-166` NcclBackend.compressed_allreduce,
the 1-bit Adam / 0-1 Adam / 1-bit LAMB communication primitive).

Two-phase, error-feedback sign compression:
  worker: x += worker_error; scale = ||x|| / sqrt(n); send sign(x) bit-packed (n/8 bytes) + one fp32 scale;
          worker_error = x - scale * sign(x)
  exchange: ONE all-to-all of the packed sign chunks (chunk r -> rank r) + all-gather of the worker scales
  server: rank r averages its chunk over the world, adds server_error, re-compresses the same way
  exchange: all-gather of the server's packed chunk + scale; every rank reconstructs the averaged tensor.
The bytes on xGMI are 1/32 of an fp32 all-reduce; all-to-all maps onto the full mesh's dedicated peer links.
Bit packing is done with vectorised tensor ops on the device.
"""
import math

import torch

from ... import comm as dist

_BITS = None


def _bit_weights(device):
    global _BITS
    if _BITS is None or _BITS.device != device:
        _BITS = (2**torch.arange(8, device=device, dtype=torch.int32)).to(torch.uint8)
    return _BITS


def pack_signs(x):
    """x [n] (n % 8 == 0) -> uint8 [n/8], bit j of byte i = (x[8i+j] >= 0)."""
    b = (x >= 0).view(-1, 8).to(torch.uint8)
    return (b * _bit_weights(x.device)).sum(dim=1, dtype=torch.uint8)


def unpack_signs(packed, dtype=torch.float32):
    """uint8 [m] -> +-1 [8m]."""
    bits = torch.bitwise_and(packed.view(-1, 1), _bit_weights(packed.device)).ne(0)
    return bits.view(-1).to(dtype).mul_(2).sub_(1)


class CompressedBackend:

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def padded_size(self, n):
        q = self.world * 8
        return int(math.ceil(n / q) * q)

    @torch.no_grad()
    def compressed_allreduce(self, buffer, worker_error, server_error):
        """Average `buffer` over the group in place with 1-bit compression. `worker_error` has buffer's padded size,
        `server_error` has padded/world elements; both persist across calls (error feedback)."""
        n = buffer.numel()
        N = worker_error.numel()
        W = self.world
        chunk = N // W
        x = torch.zeros(N, dtype=torch.float32, device=buffer.device)
        x[:n].copy_(buffer.reshape(-1))
        x.add_(worker_error)
        scale = x.norm() / math.sqrt(n)
        signs = pack_signs(x)
        worker_error.copy_(x - scale * unpack_signs(signs))
        # phase 1: chunk r of every rank's signs -> rank r; scales to everyone
        recv = torch.empty_like(signs)
        dist.all_to_all_single(recv, signs, group=self.group)
        scales = torch.empty(W, dtype=torch.float32, device=buffer.device)
        dist.all_gather_into_tensor(scales, scale.reshape(1).float(), group=self.group)
        mine = unpack_signs(recv).view(W, chunk).mul_(scales.view(W, 1)).mean(dim=0)
        mine.add_(server_error)
        s_scale = mine.norm() / math.sqrt(chunk)
        s_signs = pack_signs(mine)
        server_error.copy_(mine - s_scale * unpack_signs(s_signs))
        # phase 2: every rank's server chunk + scale to everyone
        all_signs = torch.empty(W * s_signs.numel(), dtype=torch.uint8, device=buffer.device)
        dist.all_gather_into_tensor(all_signs, s_signs, group=self.group)
        s_scales = torch.empty(W, dtype=torch.float32, device=buffer.device)
        dist.all_gather_into_tensor(s_scales, s_scale.reshape(1).float(), group=self.group)
        out = unpack_signs(all_signs).view(W, chunk).mul_(s_scales.view(W, 1)).view(-1)
        buffer.reshape(-1).copy_(out[:n].to(buffer.dtype))
        return buffer
