"""NVMe residency for the host-stepped optimizer partition (reference `runtime/swap_tensor/
partitioned_optimizer_swapper.py:29`, `pipelined_optimizer_swapper.py:51`).

The master weights ("p": fp32, or the int16 residuals of split masters) and the two fp32 Adam moments ("m", "v") of
an NVMe-resident range live in files, chunked into `chunk_numel` pieces (the ZeRO `sub_group_size`). A host step
streams them: while CPU Adam updates chunk i out of one pinned buffer set, chunk i+1 is being read into the other and
chunk i-1 written back (separate read / write aio handles), so host memory holds 2 chunk sets instead of 12 bytes per
parameter. Transfers are always whole 4 KiB multiples from page-aligned buffers so the aio engine can use O_DIRECT
(no page-cache copy of the state). `read_range` / `write_range` give the rest of the optimizer (checkpointing,
per-parameter fp32 views, elastic reload) random access.
"""
import torch

from .tensor_swapper import AsyncTensorSwapper

_IO_ALIGN = 2048  # elements: 4 KiB for the narrowest (int16) kind


class OptimizerStateSwapper:

    def __init__(self, aio_config, folder, chunk_numel=64 * 2**20, pin=True, with_master=True,
                 master_dtype=torch.float32):
        self.sw = AsyncTensorSwapper(aio_config, folder)
        self.chunk = max(_IO_ALIGN, (int(chunk_numel) + _IO_ALIGN - 1) // _IO_ALIGN * _IO_ALIGN)
        self.pin = pin
        self.with_master = with_master
        self.kinds = {"m": torch.float32, "v": torch.float32}
        if with_master:
            self.kinds["p"] = master_dtype
        self.sizes = {}       # og -> numel
        self.step_count = {}  # og -> adam step
        self._bufs = None
        self._scratch = {}

    def _chunks(self, og):
        n = self.sizes[og]
        return [(s, min(s + self.chunk, n)) for s in range(0, n, self.chunk)]

    @staticmethod
    def _io_len(n):
        return (n + _IO_ALIGN - 1) // _IO_ALIGN * _IO_ALIGN

    def _mk(self, dtype):
        """Chunk buffers only ever meet the CPU optimizer and the file system (never a device copy), so they are
        page-aligned, mlock'ed host memory from the aio engine: O_DIRECT can pin it, which it cannot do with memory
        mapped by the GPU driver (hipHostMalloc)."""
        t = self.sw.reader.new_cpu_locked_tensor(self.chunk, torch.empty(0, dtype=dtype))
        t.zero_()
        return t

    def _buffers(self):
        if self._bufs is None:
            self._bufs = [{k: self._mk(dt) for k, dt in self.kinds.items()} for _ in range(2)]
        return self._bufs

    def _scratch_buf(self, kind):
        if kind not in self._scratch:
            self._scratch[kind] = self._mk(self.kinds[kind])
        return self._scratch[kind]

    def _key(self, og, ci, kind):
        return f"og{og}_c{ci}_{kind}"

    def bytes_on_disk(self):
        return sum(self._io_len(e - s) * torch.empty(0, dtype=dt).element_size()
                   for og in self.sizes for (s, e) in self._chunks(og) for dt in self.kinds.values())

    def register(self, og, numel, master_init=None):
        """Create the files of `numel` elements of optimizer group og: zero moments and the master, filled chunk by
        chunk by `master_init(lo, hi, buffer)` (zeros without it)."""
        self.sizes[og] = int(numel)
        self.step_count[og] = 0
        for ci, (s, e) in enumerate(self._chunks(og)):
            for kind in self.kinds:
                buf = self._scratch_buf(kind)
                buf.zero_()
                if kind == "p" and master_init is not None:
                    master_init(s, e, buf[:e - s])
                self.sw.swap_out(self._key(og, ci, kind), buf[:self._io_len(e - s)], async_op=False)

    def step(self, og, update_fn, step=None):
        """Stream og through `update_fn(lo, hi, exp_avg, exp_avg_sq, step, master)` (in place; master is None
        unless with_master)."""
        self.step_count[og] = int(step) if step is not None else self.step_count[og] + 1
        chunks = self._chunks(og)
        bufs = self._buffers()

        def read(ci, slot):
            s, e = chunks[ci]
            for k in self.kinds:
                self.sw.swap_in(self._key(og, ci, k), bufs[slot][k][:self._io_len(e - s)])

        read(0, 0)
        self.sw.wait_reads()
        for ci, (s, e) in enumerate(chunks):
            slot = ci % 2
            if ci + 1 < len(chunks):
                self.sw.wait_writes()  # the other slot's previous write-back must finish before reuse
                read(ci + 1, 1 - slot)
            b = bufs[slot]
            update_fn(s, e, b["m"][:e - s], b["v"][:e - s], self.step_count[og],
                      b["p"][:e - s] if self.with_master else None)
            for k in self.kinds:
                self.sw.swap_out(self._key(og, ci, k), b[k][:self._io_len(e - s)])
            self.sw.wait_reads()
        self.sw.wait_writes()

    # ---------------------------------------------------------------- random access
    def read_range(self, og, kind, lo, hi):
        out = torch.empty(hi - lo, dtype=self.kinds[kind])
        buf = self._scratch_buf(kind)
        for ci, (s, e) in enumerate(self._chunks(og)):
            a, b = max(s, lo), min(e, hi)
            if a >= b:
                continue
            self.sw.swap_in(self._key(og, ci, kind), buf[:self._io_len(e - s)], async_op=False)
            out[a - lo:b - lo].copy_(buf[a - s:b - s])
        return out

    def write_range(self, og, kind, lo, t):
        t = t.reshape(-1).to(self.kinds[kind])
        hi = lo + t.numel()
        buf = self._scratch_buf(kind)
        for ci, (s, e) in enumerate(self._chunks(og)):
            a, b = max(s, lo), min(e, hi)
            if a >= b:
                continue
            if not (a == s and b == e):  # partial chunk: read-modify-write
                self.sw.swap_in(self._key(og, ci, kind), buf[:self._io_len(e - s)], async_op=False)
            buf[a - s:b - s].copy_(t[a - lo:b - lo])
            self.sw.swap_out(self._key(og, ci, kind), buf[:self._io_len(e - s)], async_op=False)

    def read_kind(self, og, kind):
        return self.read_range(og, kind, 0, self.sizes[og])

    # fp32-master helpers kept for callers that address the master only
    def read_master(self, og, lo, hi):
        return self.read_range(og, "p", lo, hi)

    def write_master(self, og, lo, t):
        self.write_range(og, "p", lo, t)

    def read_full(self, og):
        return self.read_kind(og, "m"), self.read_kind(og, "v"), self.step_count[og]

    def write_full(self, og, m, v, step):
        self.step_count[og] = int(step)
        self.write_range(og, "m", 0, m)
        self.write_range(og, "v", 0, v)


class NvmeFlat:
    """The NVMe-resident master of one optimizer group, with the slice / copy surface of a flat tensor."""

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
