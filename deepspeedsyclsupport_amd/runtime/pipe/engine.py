"""PipelineEngine: 1F1B pipeline-parallel training with data parallelism across pipeline replicas
(reference `runtime/pipe/engine.py:55-1371`).

`train_batch(data_iter)` runs `gradient_accumulation_steps` micro-batches through the stage's TrainSchedule and steps
the optimizer once; `eval_batch` runs the InferenceSchedule. Activations/gradients travel between neighbouring stages
with RCCL p2p (isend/irecv on the HIP stream; over xGMI when stages share a node); shapes are exchanged once as a
small int64 metadata tensor and cached. ZeRO stage <= 1 only (as in the reference, `pipe/engine.py:71-72`).
"""
import torch

from ... import comm as dist
from ...utils.logging import log_dist, logger
from ..engine import DeepSpeedEngine
from . import schedule as S
from .module import PipelineModule

_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool, torch.float64,
           torch.uint8, torch.int8]
_META_LEN = 256


def is_even(n):
    return n % 2 == 0


class PipelineEngine(DeepSpeedEngine):

    def __init__(self, has_bool_tensors=False, *super_args, **super_kwargs):
        super().__init__(*super_args, **super_kwargs)
        assert isinstance(self.module, PipelineModule), "model must be a PipelineModule"
        assert self.zero_optimization_stage() < 2, "ZeRO-2 and ZeRO-3 are incompatible with pipeline parallelism"
        self.grid = self.module._grid
        self.num_stages = self.grid.pipe_parallel_size
        self.stage_id = self.grid.get_stage_id()
        self.prev_stage = self.stage_id - 1
        self.next_stage = self.stage_id + 1
        self.micro_batches = self.gradient_accumulation_steps()
        self.is_pipe_parallel = self.num_stages > 1
        self.is_data_parallel = self.grid.data_parallel_size > 1
        self.has_bool_tensors = has_bool_tensors
        self.agg_train_loss = None
        self.total_loss = None
        self._meta_sent = {"act": False, "grad": False}
        self._recv_meta = {"act": None, "grad": None}
        self._send_works = []
        self.pipe_buffers = {"inputs": [], "labels": [], "outputs": [], "output_tensors": []}
        self.first_output_send = True
        self.loss = torch.tensor(0.0, device=self.device)
        self.data_iterator = None
        self.batch_fn = None
        self.module.checkpoint_parallel_write_pipeline = self._config.checkpoint_parallel_write_pipeline
        log_dist(f"PipelineEngine: stages={self.num_stages} stage={self.stage_id} dp={self.grid.data_parallel_size} "
                 f"micro_batches={self.micro_batches}", ranks=[-1])

    # ------------------------------------------------------------------------------------------ checkpoints
    def module_state_dict(self, destination=None, prefix="", keep_vars=False, exclude_frozen_parameters=False):
        """The stage's weights go to one file per layer, indexed by global layer number, next to the per-stage
        model-states file, which then carries no module (reference `runtime/pipe/engine.py:1324-1345`): that is what
        lets a checkpoint load under another stage count. Returns the plain dict only outside a checkpoint save."""
        path = getattr(self, "_curr_ckpt_path", None)
        if path is None:
            return super().module_state_dict(destination, prefix, keep_vars, exclude_frozen_parameters)
        self.module.save_state_dict(path, self.checkpoint_engine, exclude_frozen_params=exclude_frozen_parameters)
        return None

    def save_checkpoint(self, *args, **kwargs):
        try:
            return super().save_checkpoint(*args, **kwargs)
        finally:
            self._curr_ckpt_path = None

    def load_checkpoint(self, *args, **kwargs):
        try:
            return super().load_checkpoint(*args, **kwargs)
        finally:
            self._curr_ckpt_path = None

    @torch.no_grad()
    def _load_module_state(self, sd, strict=True):
        if sd:  # a checkpoint that carries the module inline
            return super()._load_module_state(sd, strict=strict)
        self.module.load_state_dir(self._curr_ckpt_path, self.checkpoint_engine, strict=strict)
        if self.optimizer is not None:
            self.optimizer.refresh_from_module()
        return []

    # ------------------------------------------------------------------------------------------ helpers
    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.num_stages - 1

    def set_dataiterator(self, iterator):
        self.data_iterator = iterator

    def set_batch_fn(self, fn):
        self.batch_fn = fn

    def reset_activation_shape(self):
        self._meta_sent = {"act": False, "grad": False}
        self._recv_meta = {"act": None, "grad": None}

    def _stage_rank(self, stage):
        return self.grid.stage_to_global(stage_id=stage)

    def _to_device(self, x):
        if torch.is_tensor(x):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (list, tuple)):
            return type(x)(self._to_device(t) for t in x)
        return x

    def _reserve(self, n):
        for k in self.pipe_buffers:
            while len(self.pipe_buffers[k]) < n:
                self.pipe_buffers[k].append(None)

    # ------------------------------------------------------------------------------------------ p2p with meta
    def _meta_of(self, tensors):
        meta = [len(tensors)]
        for t in tensors:
            meta += [t.dim()] + list(t.shape) + [_DTYPES.index(t.dtype), int(t.requires_grad or t.is_floating_point())]
        assert len(meta) <= _META_LEN, "too many activation tensors for the metadata buffer"
        return torch.tensor(meta + [0] * (_META_LEN - len(meta)), dtype=torch.long, device=self.device)

    @staticmethod
    def _parse_meta(meta):
        meta = meta.tolist()
        n, i, out = meta[0], 1, []
        for _ in range(n):
            nd = meta[i]
            shape = meta[i + 1:i + 1 + nd]
            dt = _DTYPES[meta[i + 1 + nd]]
            rg = bool(meta[i + 2 + nd])
            out.append((shape, dt, rg))
            i += 3 + nd
        return out

    def _send(self, tensors, dst_stage, kind):
        dst = self._stage_rank(dst_stage)
        if not self._meta_sent[kind]:
            dist.send(self._meta_of(tensors), dst)
            self._meta_sent[kind] = True
        for t in tensors:
            self._send_works.append((dist.isend(t.contiguous(), dst), t))

    def _recv(self, src_stage, kind):
        src = self._stage_rank(src_stage)
        if self._recv_meta[kind] is None:
            meta = torch.zeros(_META_LEN, dtype=torch.long, device=self.device)
            dist.recv(meta, src)
            self._recv_meta[kind] = self._parse_meta(meta)
        out = []
        for shape, dt, rg in self._recv_meta[kind]:
            buf = torch.empty(shape, dtype=dt, device=self.device)
            dist.irecv(buf, src).wait()
            out.append(buf)
        return out

    def _drain_sends(self):
        for w, _ in self._send_works:
            w.wait()
        self._send_works = []

    # ------------------------------------------------------------------------------------------ instructions
    def _exec_load_micro_batch(self, buffer_id):
        batch = self.batch_fn(next(self.data_iterator)) if self.batch_fn else next(self.data_iterator)
        batch = self._to_device(batch)
        if self.is_first_stage():
            inputs = batch[0]
            if torch.is_tensor(inputs):
                inputs = inputs.clone()
            self.pipe_buffers["inputs"][buffer_id] = inputs
        if self.is_last_stage():
            self.pipe_buffers["labels"][buffer_id] = batch[1]

    def _exec_recv_activations(self, buffer_id):
        ts = self._recv(self.prev_stage, "act")
        for t in ts:
            if t.is_floating_point():
                t.requires_grad_(True)
        self.pipe_buffers["inputs"][buffer_id] = ts[0] if len(ts) == 1 else tuple(ts)

    def _exec_forward_pass(self, buffer_id):
        inputs = self.pipe_buffers["inputs"][buffer_id]
        outputs = self.module(inputs)
        if self.is_last_stage():
            if self.module.loss_fn is not None and self._compute_loss:
                labels = self.pipe_buffers["labels"][buffer_id]
                self.loss = self.module.loss_fn(outputs, labels)
            else:
                self.loss = outputs
            if self._compute_loss:
                if self.total_loss is None:
                    self.total_loss = torch.zeros_like(self.loss.detach().float())
                self.total_loss += self.loss.detach().float()
            self.pipe_buffers["outputs"][buffer_id] = self.loss
            if self._return_outputs:
                self.fwd_outputs.append(outputs.detach() if torch.is_tensor(outputs) else outputs)
        else:
            self.pipe_buffers["outputs"][buffer_id] = outputs

    def _exec_send_activations(self, buffer_id):
        out = self.pipe_buffers["outputs"][buffer_id]
        ts = [out] if torch.is_tensor(out) else list(out)
        self._send([t.detach() for t in ts], self.next_stage, "act")

    def _exec_recv_grads(self, buffer_id):
        ts = self._recv(self.next_stage, "grad")
        self.pipe_buffers["output_tensors"][buffer_id] = ts

    def _exec_backward_pass(self, buffer_id):
        opt = self.optimizer
        out = self.pipe_buffers["outputs"][buffer_id]
        opt.is_gradient_accumulation_boundary = False  # DP reduction happens in ReduceGrads (after tied grads)
        opt.backward_prologue()
        if self.is_last_stage():
            loss = out / self.micro_batches
            if opt.dtype == torch.float16:
                loss = loss.float() * opt.loss_scale
            loss.backward()
        else:
            outs = [out] if torch.is_tensor(out) else list(out)
            grads = self.pipe_buffers["output_tensors"][buffer_id]
            pairs = [(o, g) for o, g in zip(outs, grads) if o.requires_grad]
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        opt.backward_epilogue()
        self.pipe_buffers["outputs"][buffer_id] = None
        self.pipe_buffers["output_tensors"][buffer_id] = None

    def _exec_send_grads(self, buffer_id):
        inputs = self.pipe_buffers["inputs"][buffer_id]
        ins = [inputs] if torch.is_tensor(inputs) else list(inputs)
        grads = [(t.grad if t.grad is not None else torch.zeros_like(t)) for t in ins if t.is_floating_point()]
        self._send(grads, self.prev_stage, "grad")
        self.pipe_buffers["inputs"][buffer_id] = None

    def _exec_reduce_tied_grads(self):
        self.module.allreduce_tied_weight_gradients()

    def _exec_reduce_grads(self):
        self.optimizer.reduce_gradients()

    def _exec_optimizer_step(self):
        self._drain_sends()
        self.optimizer.step()
        if not self.optimizer.overflow and self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.global_steps += 1
        self.global_samples += self.train_batch_size()

    _INSTRUCTION_MAP = {
        S.OptimizerStep: _exec_optimizer_step,
        S.ReduceGrads: _exec_reduce_grads,
        S.ReduceTiedGrads: _exec_reduce_tied_grads,
        S.LoadMicroBatch: _exec_load_micro_batch,
        S.ForwardPass: _exec_forward_pass,
        S.BackwardPass: _exec_backward_pass,
        S.SendActivation: _exec_send_activations,
        S.RecvActivation: _exec_recv_activations,
        S.SendGrad: _exec_send_grads,
        S.RecvGrad: _exec_recv_grads,
    }

    def _exec_schedule(self, sched):
        self._reserve(sched.num_pipe_buffers())
        for step_cmds in sched:
            for cmd in step_cmds:
                fn = self._INSTRUCTION_MAP[type(cmd)]
                if isinstance(cmd, S.BufferOpInstruction):
                    fn(self, cmd.buffer_id)
                else:
                    fn(self)

    # ------------------------------------------------------------------------------------------ public API
    def train_batch(self, data_iter=None):
        if data_iter is not None:
            self.set_dataiterator(data_iter)
        self.module.train()
        self.total_loss = None
        self._compute_loss = True
        self._return_outputs = False
        sched = S.TrainSchedule(micro_batches=self.micro_batches, stages=self.num_stages, stage_id=self.stage_id)
        self._exec_schedule(sched)
        self._drain_sends()
        self.agg_train_loss = self._aggregate_total_loss()
        return self.agg_train_loss

    @torch.no_grad()
    def eval_batch(self, data_iter, return_logits=False, compute_loss=True, reduce_output="avg", bcast_loss=True,
                   num_micro_batches=None):
        self.module.eval()
        self.set_dataiterator(data_iter)
        self.total_loss = None
        self._compute_loss = compute_loss
        self._return_outputs = return_logits
        self.fwd_outputs = []
        mb = num_micro_batches or self.micro_batches
        sched = S.InferenceSchedule(micro_batches=mb, stages=self.num_stages, stage_id=self.stage_id)
        self._exec_schedule(sched)
        self._drain_sends()
        loss = self._aggregate_total_loss(mb) if compute_loss else None
        self.module.train()
        if return_logits:
            return loss, self.fwd_outputs
        return loss

    def _aggregate_total_loss(self, micro_batches=None):
        mb = micro_batches or self.micro_batches
        last = self._stage_rank(self.num_stages - 1)
        if self.is_last_stage():
            loss = (self.total_loss / mb) if self.total_loss is not None else torch.zeros((), device=self.device)
            if self.is_data_parallel:
                dist.all_reduce(loss, group=self.grid.get_data_parallel_group())
                loss /= self.grid.data_parallel_size
            t = loss.clone().float().reshape(1)
        else:
            t = torch.zeros(1, device=self.device)
        if self.is_pipe_parallel:
            dist.broadcast(t, src=last, group=self.grid.get_pipe_parallel_group())
        return t[0]

    def set_dataloader(self, loader):
        """Stages that read data (first: inputs, last: labels) iterate `loader` (reference `pipe/engine.py:584`)."""
        if self.is_first_stage() or self.is_last_stage():
            self.training_dataloader = loader
            self.data_iterator = iter(loader)

    def set_has_attention_mask(self, value):
        assert isinstance(value, bool)
        self.has_attention_mask = value

    def set_train_batch_size(self, train_batch_size):
        """New global batch at the same micro-batch size: the number of micro-batches per step follows."""
        super().set_train_batch_size(train_batch_size)
        self.micro_batches = self.gradient_accumulation_steps()

    def log_for_device(self, *msg):
        if self.global_rank == 0:
            logger.info(f"RANK={self.global_rank} PIPE-ID={self.stage_id} DATA-ID={self.grid.data_parallel_id} "
                        + " ".join(str(m) for m in msg))

    def mem_status(self, msg, print_rank=-1, reset_max=False):
        """Device memory now / peak in GiB (reference `pipe/engine.py:1263-1300`)."""
        if print_rank != -1 and self.global_rank != print_rank:
            return
        if self.device.type != "cuda":
            return
        torch.cuda.synchronize()
        if reset_max:
            torch.cuda.reset_peak_memory_stats()
        gib = 1024**3
        logger.info(f"RANK={self.global_rank} STAGE={self.stage_id} MEMSTATS {msg} "
                    f"current alloc={torch.cuda.memory_allocated() / gib:.4f}GB "
                    f"max alloc={torch.cuda.max_memory_allocated() / gib:.4f}GB "
                    f"current cache={torch.cuda.memory_reserved() / gib:.4f}GB")

    def tput_log(self, *msg):
        if self.global_rank == 0 and self.tput_timer is not None:
            logger.info(f"steps: {self.global_steps} samples/sec: {self.tput_timer.avg_samples_per_sec():.3f} "
                        + " ".join(str(m) for m in msg))

    def forward(self, *args, **kwargs):
        raise RuntimeError("Only train_batch() / eval_batch() are accessible in pipeline mode.")

    def backward(self, *args, **kwargs):
        raise RuntimeError("Only train_batch() is accessible in pipeline mode.")

    def step(self, *args, **kwargs):
        raise RuntimeError("Only train_batch() is accessible in pipeline mode.")
