"""Host / NVMe residency of optimizer state and the transfer pipelines around it: ZeRO-Offload, ZeRO-Offload++
Twin-Flow and ZeRO-Infinity for the flat-group optimizer.

Reference behaviour: `runtime/zero/stage3.py:198-211,808-817,926-942` (Twin-Flow: a `ratio` of the sub-groups is
stepped by CPU Adam, the rest by the device optimizer), `stage3.py:1389-1407` (gradients copied to pinned host
memory during backward), `csrc/adam/cpu_adam_impl.cpp:58-112` (the host update writes the 16-bit weights into a
pinned buffer and copies them up on side streams), `runtime/swap_tensor/partitioned_optimizer_swapper.py:29`
(optimizer state on NVMe).

MI355X design. Per optimizer group the offloaded elements form ONE flat "offloaded space" of `n[og]` elements; its
first `resident[og]` elements keep their state in host DRAM, the tail lives on NVMe and is streamed in chunks. For
every element the host holds
    fp32 master (4 B)   or, with split masters, a 16-bit residual (2 B): master bits = (bf16 weight << 16) + residual
    two fp32 moments (8 B)
    one 16-bit staging slot (2 B, pinned): the gradient travels down into it and the updated weight back up out of it
so a parameter costs 14 B (12 B split) of host memory and nothing on the device beyond its 16-bit weight.

Three copy engines run next to the compute stream:
  * `d2h` stream — as soon as a gradient (or a reduce-scattered gradient segment) is final in backward it is copied
    into its staging slot and the device copy is freed; its sum of squares is taken on the device first, so the
    global norm needs no second pass. In-flight bytes are bounded so a fast backward cannot pile up gradients.
  * a worker thread — after the clip coefficient is known it walks the pieces in forward order: CPU Adam (native,
    AVX-512/OpenMP, interpreter lock released) on one piece while
  * `h2d` stream — the previous piece's updated 16-bit weights are copied back into the shard, each followed by an
    event. `wait()` joins everything; with `overlap_forward` the next forward instead waits per module, so the host
    update of late layers overlaps the forward of early ones.
The device part of the optimizer state is stepped by the fused HIP Adam on the main thread at the same time.
"""
import queue
import threading

import torch

from ...utils.logging import logger


def split_join(hi, lo):
    """fp32 master from a bf16 weight tensor `hi` and its int16 residual `lo` (same device, same numel)."""
    u = (hi.view(torch.int16).to(torch.int32) << 16) + lo.to(torch.int32)
    return u.view(torch.float32)


def split_cut(f32):
    """(bf16 weight, int16 residual) of fp32 values: weight = value rounded to nearest, ties away from zero."""
    u = f32.contiguous().view(torch.int32)
    hi = ((u + 0x8000) >> 16).to(torch.int16).view(torch.bfloat16)
    lo = (u & 0xffff).to(torch.int16)  # values >= 0x8000 wrap to the negative residuals
    return hi, lo


def _round_up(n, k):
    return (n + k - 1) // k * k


class _Piece:
    """A contiguous range of one optimizer group's offloaded space backed by a slice of a flat group's shard."""
    __slots__ = ("og", "moff", "n", "group", "s", "alpha", "covered", "accumulated", "flag", "event")

    def __init__(self, og, moff, n, group, s):
        self.og, self.moff, self.n, self.group, self.s = og, moff, n, group, s
        self.alpha = 1.0
        self.covered = []          # [(offset in piece, numel)] gradient ranges staged this step
        self.accumulated = False   # gradients live in the fp32 host accumulator (gas > 1), not in the staging slot
        self.flag = threading.Event()
        self.flag.set()
        self.event = None


class OffloadedState:
    MAX_INFLIGHT_BYTES = 16 << 30

    def __init__(self, opt, sizes, resident, split, pin, swapper, overlap_forward=False):
        self.opt = opt
        self.dtype = opt.dtype
        self.device = opt.device
        self.cuda = self.device.type == "cuda"
        self.n = list(sizes)
        self.res = [min(r, n) for r, n in zip(resident, sizes)]
        self.split = bool(split)
        self.pin = bool(pin) and self.cuda
        self.swapper = swapper
        self.overlap_forward = bool(overlap_forward) and self.cuda
        nog = len(sizes)
        self.master = [None] * nog   # fp32 [res] (or int16 residuals when split)
        self.m = [None] * nog
        self.v = [None] * nog
        self.stage = [None] * nog    # 16-bit [n] (pinned): gradient in, weight out
        self.acc = [None] * nog      # fp32 [n] gradient accumulator (gas > 1 only)
        self.step_count = [0] * nog
        self.pieces = [[] for _ in range(nog)]
        self.all_pieces = []
        self.by_group = {}
        mdt = torch.int16 if self.split else torch.float32
        for og in range(nog):
            if self.n[og] == 0:
                continue
            self.master[og] = torch.zeros(self.res[og], dtype=mdt)
            self.stage[og] = self._host(self.n[og], self.dtype)
            if self.n[og] > self.res[og]:
                assert swapper is not None, "offloaded elements beyond the resident part need an NVMe swapper"
        self.d2h = torch.cuda.Stream() if self.cuda else None
        self.h2d = torch.cuda.Stream() if self.cuda else None
        self._inflight = []          # (event, bytes) of staged gradient copies
        self._inflight_bytes = 0
        self._sq = {}                # og -> sum of squares (scaled by alpha^2) of the gradients staged this step
        self._bounce = None
        self._acc_bounce = None
        self._acc_slot = 0
        self._worker = None
        self._jobs = queue.Queue()
        self._err = None
        if self.overlap_forward:
            # worker and main thread both run short Python sections between native calls; a short switch interval
            # keeps either from waiting whole 5 ms slices for the interpreter lock
            import sys
            sys.setswitchinterval(min(sys.getswitchinterval(), 2e-4))

    # ---------------------------------------------------------------- allocation
    def _host(self, n, dtype):
        if self.pin:
            from ...ops.native import hip_ops
            return hip_ops().alloc_pinned(int(n), dtype)  # exact size (torch's pinned pool rounds up to 2^k)
        return torch.empty(int(n), dtype=dtype)

    def add_piece(self, og, moff, n, group, s):
        p = _Piece(og, moff, n, group, s)
        self.pieces[og].append(p)
        return p

    def finalize(self):
        """Order of the host step: groups without a module first (their weights are needed before any module's
        pre-forward hook can wait), then modules in registration (= forward) order."""
        for og in range(len(self.n)):
            self.pieces[og].sort(key=lambda p: p.moff)
        self.all_pieces = sorted((p for ps in self.pieces for p in ps),
                                 key=lambda p: (p.group.module is not None, p.group.idx, p.moff))
        self.by_group = {}
        for p in self.all_pieces:
            self.by_group.setdefault(p.group.idx, []).append(p)

    def host_bytes(self):
        per = (2 if self.split else 4) + 8
        return sum(r * per + n * self.stage[og].element_size()
                   for og, (n, r) in enumerate(zip(self.n, self.res)) if n)

    # ---------------------------------------------------------------- master init / range access
    @torch.no_grad()
    def init_master(self, piece):
        """Masters start as the exact 16-bit weights (residual 0 when split)."""
        if self.split:
            return
        og, lo, hi = piece.og, piece.moff, piece.moff + piece.n
        r = self.res[og]
        if lo < r:
            k = min(hi, r) - lo
            self.master[og][lo:lo + k].copy_(piece.group.shard[piece.s:piece.s + k])

    def nvme_master_init(self, og):
        """Fill callback for the swapper: chunk [a, b) of og's NVMe tail (tail coordinates) from the shards."""
        base = self.res[og]

        def init(a, b, buf):
            buf.zero_()
            if self.split:
                return
            for p in self.pieces[og]:
                x0, x1 = max(p.moff, base + a), min(p.moff + p.n, base + b)
                if x0 < x1:
                    buf[x0 - base - a:x1 - base - a].copy_(p.group.shard[p.s + x0 - p.moff:p.s + x1 - p.moff])
        return init

    _KIND = {"fp32": "p", "residual": "p", "exp_avg": "m", "exp_avg_sq": "v"}

    def _resident(self, key, og):
        return {"p": self.master, "m": self.m, "v": self.v}[self._KIND[key]][og]

    def read_state(self, og, key, lo, hi):
        """Host tensor with `key` ('fp32' master / 'residual' of split masters, 'exp_avg', 'exp_avg_sq') over the
        offloaded range [lo, hi) of og; None for moments that do not exist yet."""
        self.wait()
        if key in ("exp_avg", "exp_avg_sq") and self.step_count[og] == 0 and self.m[og] is None:
            return None
        r = self.res[og]
        src = self._resident(key, og)
        parts = []
        if lo < r:
            parts.append(src[lo:min(hi, r)])
        if hi > r:
            parts.append(self.swapper.read_range(og, self._KIND[key], max(lo, r) - r, hi - r))
        return parts[0] if len(parts) == 1 else torch.cat(parts)

    def write_state(self, og, key, lo, values):
        self.wait()
        if key in ("exp_avg", "exp_avg_sq"):
            self._ensure_moments(og)
        r = self.res[og]
        hi = lo + values.numel()
        dst = self._resident(key, og)
        values = values.reshape(-1).to("cpu")
        if lo < r:
            k = min(hi, r) - lo
            dst[lo:lo + k].copy_(values[:k])
        if hi > r:
            a = max(lo, r)
            self.swapper.write_range(og, self._KIND[key], a - r, values[a - lo:])

    def _ensure_moments(self, og):
        if self.m[og] is None and self.n[og]:
            self.m[og] = torch.zeros(self.res[og], dtype=torch.float32)
            self.v[og] = torch.zeros(self.res[og], dtype=torch.float32)

    # ---------------------------------------------------------------- gradient staging (backward)
    def _add_sq(self, og, sq):
        self._sq[og] = sq if og not in self._sq else self._sq[og] + sq

    @torch.no_grad()
    def stage_grad(self, piece, src, alpha, accumulate=False, off=0):
        """`src` (device or host 1-D tensor) is the final gradient of piece elements [off, off + numel) for this
        micro-step; `alpha` is the factor still to be applied to it. With `accumulate` (micro-steps of a gas > 1
        window under partitioned ZeRO-2/3) it is summed into the fp32 host accumulator instead."""
        og, n = piece.og, src.numel()
        lo = piece.moff + off
        piece.alpha = alpha
        if accumulate or piece.accumulated:
            self._accumulate(piece, src, alpha, off)
            return
        piece.covered.append((off, n))
        dst = self.stage[og][lo:lo + n]
        if not (self.cuda and src.is_cuda):
            dst.copy_(src)
            self._add_sq(og, src.float().pow(2).sum() * (alpha * alpha))
            return
        from ...ops import native
        src = src if src.is_contiguous() else src.contiguous()
        sq = native.hip_ops().sumsq_multi([src])
        self._add_sq(og, sq * (alpha * alpha) if alpha != 1.0 else sq)
        self._throttle(n * src.element_size())
        self.d2h.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.d2h):
            dst.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.d2h)
        src.record_stream(self.d2h)
        self._inflight.append((ev, n * src.element_size()))
        self._inflight_bytes += n * src.element_size()

    def _throttle(self, incoming):
        """Bound the gradient bytes waiting for their copy down, so backward cannot run arbitrarily far ahead of
        the link and hold all of them in device memory."""
        while self._inflight and self._inflight[0][0].query():
            self._inflight_bytes -= self._inflight.pop(0)[1]
        while self._inflight and self._inflight_bytes + incoming > self.MAX_INFLIGHT_BYTES:
            ev, b = self._inflight.pop(0)
            ev.synchronize()
            self._inflight_bytes -= b

    def _accumulate(self, piece, src, alpha, off):
        from ...ops.native import cpu_ops
        og, n = piece.og, src.numel()
        lo = piece.moff + off
        if self.acc[og] is None:
            self.acc[og] = torch.zeros(self.n[og], dtype=torch.float32)
        dst = self.acc[og][lo:lo + n]
        first = (off, n) not in piece.covered
        if first:
            piece.covered.append((off, n))
        piece.accumulated = True
        piece.alpha = 1.0  # alpha is folded into the accumulator
        if not (self.cuda and src.is_cuda):
            cpu_ops().cpu_accumulate(dst, src.contiguous(), alpha, first)
            return
        if self._acc_bounce is None:
            cap = max(p.n for p in self.all_pieces)
            self._acc_bounce = [(self._host(cap, self.dtype), threading.Event()) for _ in range(2)]
            for _, f in self._acc_bounce:
                f.set()
        buf, free = self._acc_bounce[self._acc_slot]
        self._acc_slot ^= 1
        free.wait()
        free.clear()
        self.d2h.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.d2h):
            buf[:n].copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.d2h)
        src.record_stream(self.d2h)

        def job():
            ev.synchronize()
            cpu_ops().cpu_accumulate(dst, buf[:n], alpha, first)
            free.set()
        self._submit(job)

    def staged_norm_sq(self):
        """og -> sum of squares of everything staged this step (device scalar, host scalar or float)."""
        out = dict(self._sq)
        acc_ogs = {p.og for p in self.all_pieces if p.accumulated}
        if acc_ogs:
            from ...ops.native import cpu_ops
            self._drain()
            for og in acc_ogs:
                tot = 0.0
                for p in self.pieces[og]:
                    if p.accumulated:
                        for (o, n) in p.covered:
                            tot += cpu_ops().cpu_sumsq(self.acc[og][p.moff + o:p.moff + o + n])
                out[og] = out[og] + tot if og in out else tot
        return out

    def discard(self):
        """Forget the gradients staged for a skipped (overflowed) step."""
        self._drain()
        if self.cuda:
            self.d2h.synchronize()
        for p in self.all_pieces:
            p.covered = []
            p.accumulated = False
        self._sq = {}
        self._inflight, self._inflight_bytes = [], 0

    # ---------------------------------------------------------------- worker plumbing
    def _submit(self, fn):
        if not self.cuda:
            fn()
            return
        if self._worker is None:
            dev = torch.cuda.current_device()

            def loop():
                torch.cuda.set_device(dev)
                if self.overlap_forward:
                    # the main thread keeps launching the next forward while this thread steps: leave it a core
                    from ...ops.native import cpu_ops
                    cpu_ops().cpu_set_omp_threads(max(1, cpu_ops().cpu_get_omp_threads() - 1))
                while True:
                    f = self._jobs.get()
                    if f is None:
                        return
                    try:
                        f()
                    except BaseException as e:  # surfaced by wait()
                        self._err = e
                        for p in getattr(self, "all_pieces", []):
                            p.flag.set()
                    finally:
                        self._jobs.task_done()
            self._worker = threading.Thread(target=loop, daemon=True, name="ds-offload")
            self._worker.start()
        self._jobs.put(fn)

    def _drain(self):
        if self._worker is not None:
            self._jobs.join()
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError("offload worker failed") from e

    def wait(self):
        """Join the host step and make the compute stream wait for the weight copies."""
        self._drain()
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.h2d)

    def wait_group(self, g):
        """Pre-forward wait for one flat group (overlap_forward): block until its pieces' copies are issued, then
        order the compute stream after them."""
        for p in self.by_group.get(g.idx, ()):
            p.flag.wait()
            if p.event is not None:
                torch.cuda.current_stream().wait_event(p.event)
        if self._err is not None:
            self._drain()

    # ---------------------------------------------------------------- the host step
    def step(self, grad_scale, hyper):
        """Start the host update of every piece that received gradients. `hyper[og]` = dict(lr, betas, eps,
        weight_decay, bias_correction, adamw). On a GPU this returns at once (worker thread): call `wait()` (or
        rely on `wait_group`) before the weights are used."""
        todo = [p for p in self.all_pieces if p.covered]
        for og in {p.og for p in todo}:
            self._ensure_moments(og)
            self.step_count[og] += 1
        for p in todo:
            p.flag.clear()
            p.event = None
        self._sq = {}
        self._inflight, self._inflight_bytes = [], 0

        def run():
            if self.cuda:
                self.d2h.synchronize()  # every staged gradient has landed
            for p in todo:              # parameters that produced no gradient this step count as zero gradient
                self._zero_gaps(p)
            self._run_resident([p for p in todo if p.moff < self.res[p.og]], grad_scale, hyper)
            for og in sorted({p.og for p in todo if p.moff + p.n > self.res[p.og]}):
                self._run_nvme(og, [p for p in self.pieces[og] if p.covered], grad_scale, hyper)
            for p in todo:
                p.covered = []
                p.accumulated = False
                p.flag.set()
        self._submit(run)

    def _zero_gaps(self, p):
        buf = (self.acc if p.accumulated else self.stage)[p.og]
        pos = 0
        for (o, n) in sorted(p.covered):
            if o > pos:
                buf[p.moff + pos:p.moff + o].zero_()
            pos = max(pos, o + n)
        if pos < p.n:
            buf[p.moff + pos:p.moff + p.n].zero_()

    def _adam(self, og, lo, hi, master, m, v, grad, hi_in, out, scale, hyper):
        from ...ops.native import cpu_ops
        h = hyper[og]
        b1, b2 = h["betas"]
        if self.split:
            cpu_ops().cpu_adam_update_split(master, m, v, grad, hi_in, out, self.step_count[og], h["lr"], b1, b2,
                                            h["eps"], h["weight_decay"], h["bias_correction"], h["adamw"], scale)
        else:
            cpu_ops().cpu_adam_update(master, m, v, grad, out, self.step_count[og], h["lr"], b1, b2, h["eps"],
                                      h["weight_decay"], h["bias_correction"], h["adamw"], scale)

    def _grad_src(self, p, lo, hi):
        return (self.acc if p.accumulated else self.stage)[p.og][lo:hi]

    def _bounce_buffers(self, cap):
        if self._bounce is None or self._bounce[0].numel() < cap:
            self._bounce = [self._host(cap, self.dtype) for _ in range(2)]
        return self._bounce

    def _fetch_hi(self, piece, a, b, buf):
        """Copy the 16-bit weights of piece range [a, b) (offloaded-space coordinates) into buf[:b-a]."""
        src = piece.group.shard[piece.s + a - piece.moff:piece.s + b - piece.moff]
        if self.cuda and src.is_cuda:
            with torch.cuda.stream(self.d2h):
                buf[:b - a].copy_(src, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.d2h)
            return ev
        buf[:b - a].copy_(src)
        return None

    def _push(self, piece, a, b):
        """Copy updated weights stage[a:b] back into the piece's shard on the h2d stream."""
        dst = piece.group.shard[piece.s + a - piece.moff:piece.s + b - piece.moff]
        src = self.stage[piece.og][a:b]
        if self.cuda and dst.is_cuda:
            with torch.cuda.stream(self.h2d):
                dst.copy_(src, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.h2d)
            return ev
        dst.copy_(src)
        return None

    def _run_resident(self, todo, grad_scale, hyper):
        """Pieces whose state is in DRAM, in forward order; split masters prefetch the next piece's weights."""
        parts = []
        for p in todo:
            r = self.res[p.og]
            parts.append((p, p.moff, min(p.moff + p.n, r)))
        bufs = self._bounce_buffers(max((b - a for _, a, b in parts), default=0)) if self.split and parts else None
        nxt = self._fetch_hi(parts[0][0], parts[0][1], parts[0][2], bufs[0]) if bufs else None
        for i, (p, a, b) in enumerate(parts):
            og = p.og
            hi_in = None
            if bufs:
                ev, cur = nxt, bufs[i % 2]
                if i + 1 < len(parts):
                    q, qa, qb = parts[i + 1]
                    nxt = self._fetch_hi(q, qa, qb, bufs[(i + 1) % 2])
                if ev is not None:
                    ev.synchronize()
                hi_in = cur[:b - a]
            st = self.stage[og][a:b]
            self._adam(og, a, b, self.master[og][a:b], self.m[og][a:b], self.v[og][a:b], self._grad_src(p, a, b),
                       hi_in, st, grad_scale * p.alpha, hyper)
            ev = self._push(p, a, b)
            if b == p.moff + p.n:  # wholly resident: done (pieces reaching into the NVMe tail finish there)
                p.event = ev
                p.flag.set()

    def _run_nvme(self, og, pieces, grad_scale, hyper):
        base = self.res[og]
        bufs = self._bounce_buffers(self.swapper.chunk) if self.split else None

        def upd(a, b, m, v, step, master):
            # chunk [a, b) of the tail = offloaded range [base + a, base + b)
            last_ev = None
            for p in pieces:
                x0, x1 = max(p.moff, base + a), min(p.moff + p.n, base + b)
                if x0 >= x1:
                    continue
                sl = slice(x0 - base - a, x1 - base - a)
                hi_in = None
                if bufs:
                    ev = self._fetch_hi(p, x0, x1, bufs[0])
                    if ev is not None:
                        ev.synchronize()
                    hi_in = bufs[0][:x1 - x0]
                self._adam(og, x0, x1, master[sl], m[sl], v[sl], self._grad_src(p, x0, x1), hi_in,
                           self.stage[og][x0:x1], grad_scale * p.alpha, hyper)
                last_ev = self._push(p, x0, x1)
                if x1 == p.moff + p.n:
                    p.event = last_ev
                    p.flag.set()
        self.swapper.step(og, upd, step=self.step_count[og])

    # ---------------------------------------------------------------- checkpoint helpers
    def full_state(self, og):
        """(master fp32 or int16 residuals, exp_avg, exp_avg_sq, step) of og's whole offloaded space on the host."""
        self.wait()
        n = self.n[og]
        self._ensure_moments(og)
        outs = []
        for key in ("residual" if self.split else "fp32", "exp_avg", "exp_avg_sq"):
            t = self.read_state(og, key, 0, n)
            outs.append(t.clone() if t is not None else torch.zeros(n, dtype=torch.float32))
        return outs[0], outs[1], outs[2], self.step_count[og]

    def close(self):
        if self._worker is not None:
            self._drain()
            self._jobs.put(None)
            self._worker = None
