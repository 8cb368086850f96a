"""NVMe residency for the host-stepped optimizer partition (reference `runtime/swap_tensor/
partitioned_optimizer_swapper.py:29`, `pipelined_optimizer_swapper.py:51`).

The fp32 master weights (with_master) and Adam moments of the host-stepped (offloaded) optimizer partition live in
files on NVMe, chunked into `chunk_numel` pieces (the ZeRO `sub_group_size`). A host step streams them: while CPU
Adam updates chunk i out of one pinned buffer set, chunk i+1 is being read into the other and chunk i-1 written back
(separate read / write aio handles), so host memory holds 2 chunk sets instead of 12 bytes per parameter; only the
fp32 gradient accumulator and the low-precision copy stay resident. `NvmeFlat` gives the rest of the optimizer
(checkpointing, per-parameter fp32 views, elastic reload) range reads and writes of the master.
"""
import torch

from .tensor_swapper import AsyncTensorSwapper


class OptimizerStateSwapper:

    def __init__(self, aio_config, folder, chunk_numel=64 * 2**20, pin=True, with_master=False):
        self.sw = AsyncTensorSwapper(aio_config, folder)
        self.chunk = int(chunk_numel)
        self.pin = pin
        self.with_master = with_master
        self.kinds = ("m", "v", "p") if with_master else ("m", "v")
        self.sizes = {}       # og -> numel
        self.step_count = {}  # og -> adam step
        self._bufs = None

    def _chunks(self, og):
        n = self.sizes[og]
        return [(s, min(s + self.chunk, n)) for s in range(0, n, self.chunk)]

    def _buffers(self):
        if self._bufs is None:
            mk = lambda: torch.zeros(self.chunk, dtype=torch.float32, pin_memory=self.pin)  # noqa: E731
            self._bufs = [tuple(mk() for _ in self.kinds) for _ in range(2)]
        return self._bufs

    def register(self, og, numel, master_init=None):
        """Create the files of `numel` host-stepped elements of optimizer group og: zero moments and (with_master)
        the fp32 master, filled chunk by chunk by `master_init(lo, hi, buffer)`."""
        self.sizes[og] = int(numel)
        self.step_count[og] = 0
        buf = self._buffers()[0][0]
        for ci, (s, e) in enumerate(self._chunks(og)):
            buf.zero_()
            for kind in ("m", "v"):
                self.sw.swap_out(f"og{og}_c{ci}_{kind}", buf[:e - s], async_op=False)
            if self.with_master:
                if master_init is not None:
                    master_init(s, e, buf[:e - s])
                self.sw.swap_out(f"og{og}_c{ci}_p", buf[:e - s], async_op=False)

    def step(self, og, update_fn):
        """Stream og through `update_fn(lo, hi, exp_avg, exp_avg_sq, step, master)` (in place; master is None
        unless with_master)."""
        self.step_count[og] += 1
        chunks = self._chunks(og)
        bufs = self._buffers()
        key = lambda ci, k: f"og{og}_c{ci}_{k}"  # noqa: E731

        def read(ci, slot):
            s, e = chunks[ci]
            for k, b in zip(self.kinds, bufs[slot]):
                self.sw.swap_in(key(ci, k), b[:e - s])

        read(0, 0)
        self.sw.wait_reads()
        for ci, (s, e) in enumerate(chunks):
            slot = ci % 2
            if ci + 1 < len(chunks):
                self.sw.wait_writes()  # the other slot's previous write-back must finish before reuse
                read(ci + 1, 1 - slot)
            t = [b[:e - s] for b in bufs[slot]]
            update_fn(s, e, t[0], t[1], self.step_count[og], t[2] if self.with_master else None)
            for k, b in zip(self.kinds, t):
                self.sw.swap_out(key(ci, k), b)
            self.sw.wait_reads()
        self.sw.wait_writes()

    # ---------------------------------------------------------------- fp32 master range access (with_master)
    def read_master(self, og, lo, hi):
        out = torch.empty(hi - lo, dtype=torch.float32)
        for ci, (s, e) in enumerate(self._chunks(og)):
            a, b = max(s, lo), min(e, hi)
            if a >= b:
                continue
            if a == s and b == e:
                self.sw.swap_in(f"og{og}_c{ci}_p", out[a - lo:b - lo], async_op=False)
            else:
                tmp = torch.empty(e - s, dtype=torch.float32)
                self.sw.swap_in(f"og{og}_c{ci}_p", tmp, async_op=False)
                out[a - lo:b - lo].copy_(tmp[a - s:b - s])
        return out

    def write_master(self, og, lo, t):
        t = t.reshape(-1).float()
        hi = lo + t.numel()
        for ci, (s, e) in enumerate(self._chunks(og)):
            a, b = max(s, lo), min(e, hi)
            if a >= b:
                continue
            if a == s and b == e:
                self.sw.swap_out(f"og{og}_c{ci}_p", t[a - lo:b - lo].contiguous(), async_op=False)
            else:  # partial chunk: read-modify-write
                tmp = torch.empty(e - s, dtype=torch.float32)
                self.sw.swap_in(f"og{og}_c{ci}_p", tmp, async_op=False)
                tmp[a - s:b - s].copy_(t[a - lo:b - lo])
                self.sw.swap_out(f"og{og}_c{ci}_p", tmp, async_op=False)

    def read_full(self, og):
        n = self.sizes[og]
        m, v = torch.empty(n, dtype=torch.float32), torch.empty(n, dtype=torch.float32)
        for ci, (s, e) in enumerate(self._chunks(og)):
            self.sw.swap_in(f"og{og}_c{ci}_m", m[s:e], async_op=False)
            self.sw.swap_in(f"og{og}_c{ci}_v", v[s:e], async_op=False)
        return m, v, self.step_count[og]

    def write_full(self, og, m, v, step):
        self.step_count[og] = int(step)
        for ci, (s, e) in enumerate(self._chunks(og)):
            self.sw.swap_out(f"og{og}_c{ci}_m", m[s:e].contiguous().float(), async_op=False)
            self.sw.swap_out(f"og{og}_c{ci}_v", v[s:e].contiguous().float(), async_op=False)


class NvmeFlat:
    """The NVMe-resident fp32 master of one optimizer group, with the slice / copy surface the optimizer uses."""

    def __init__(self, swapper, og, numel):
        self.sw, self.og, self.n = swapper, og, int(numel)

    def numel(self):
        return self.n

    @property
    def shape(self):
        return torch.Size([self.n])

    def __getitem__(self, sl):
        lo, hi, _ = sl.indices(self.n)
        return self.sw.read_master(self.og, lo, hi)

    def write(self, lo, t):
        self.sw.write_master(self.og, lo, t)

    def read_full(self):
        return self.sw.read_master(self.og, 0, self.n)

    def copy_(self, t):
        self.sw.write_master(self.og, 0, t)
        return self
