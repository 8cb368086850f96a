"""NVMe residency for the host-side Adam moments (reference `runtime/swap_tensor/partitioned_optimizer_swapper.py:29`,
`pipelined_optimizer_swapper.py:51`).

The fp32 Adam moments of the host-stepped (offloaded) optimizer partition live in files on NVMe, chunked into
`chunk_numel` pieces. A host step streams them: while CPU Adam updates chunk i out of one pinned buffer pair, chunk
i+1 is being read into the other and chunk i-1 written back (separate read / write aio handles), so host memory
for moments is 2 x 2 chunks instead of 8 bytes per parameter.
"""
import torch

from .tensor_swapper import AsyncTensorSwapper


class OptimizerStateSwapper:

    def __init__(self, aio_config, folder, chunk_numel=64 * 2**20, pin=True):
        self.sw = AsyncTensorSwapper(aio_config, folder)
        self.chunk = int(chunk_numel)
        self.pin = pin
        self.sizes = {}       # og -> numel
        self.step_count = {}  # og -> adam step
        self._bufs = None

    def _chunks(self, og):
        n = self.sizes[og]
        return [(s, min(s + self.chunk, n)) for s in range(0, n, self.chunk)]

    def _buffers(self):
        if self._bufs is None:
            mk = lambda: torch.zeros(self.chunk, dtype=torch.float32, pin_memory=self.pin)  # noqa: E731
            self._bufs = [(mk(), mk()), (mk(), mk())]
        return self._bufs

    def register(self, og, numel):
        """Create zero-initialised moment files for `numel` host-stepped elements of optimizer group og."""
        self.sizes[og] = int(numel)
        self.step_count[og] = 0
        m, _ = self._buffers()[0]
        m.zero_()
        for ci, (s, e) in enumerate(self._chunks(og)):
            for kind in ("m", "v"):
                self.sw.swap_out(f"og{og}_c{ci}_{kind}", m[:e - s], async_op=False)

    def step(self, og, update_fn):
        """Stream the moments of og through `update_fn(lo, hi, exp_avg, exp_avg_sq, step)` (in place)."""
        self.step_count[og] += 1
        chunks = self._chunks(og)
        bufs = self._buffers()
        key = lambda ci, k: f"og{og}_c{ci}_{k}"  # noqa: E731

        def read(ci, slot):
            s, e = chunks[ci]
            self.sw.swap_in(key(ci, "m"), bufs[slot][0][:e - s])
            self.sw.swap_in(key(ci, "v"), bufs[slot][1][:e - s])

        read(0, 0)
        self.sw.wait_reads()
        for ci, (s, e) in enumerate(chunks):
            slot = ci % 2
            if ci + 1 < len(chunks):
                self.sw.wait_writes()  # the other slot's previous write-back must finish before reuse
                read(ci + 1, 1 - slot)
            m, v = bufs[slot][0][:e - s], bufs[slot][1][:e - s]
            update_fn(s, e, m, v, self.step_count[og])
            self.sw.swap_out(key(ci, "m"), m)
            self.sw.swap_out(key(ci, "v"), v)
            self.sw.wait_reads()
        self.sw.wait_writes()

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
