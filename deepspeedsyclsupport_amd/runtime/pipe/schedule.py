"""Pipeline schedules as instruction streams (reference `runtime/pipe/schedule.py:135-494`).

`TrainSchedule` is synchronous 1F1B: stage s runs min(S-s-1, M) warm-up forwards, then alternates one forward and
one backward, then drains the remaining backwards, and finally reduces tied/DP gradients and steps. Every
communication is expressed next to the compute that produces/consumes it; the engine issues sends as non-blocking
p2p (RCCL over xGMI between neighbouring stages) and receives as blocking, which is deadlock-free for this order.
`InferenceSchedule` is a forward-only pipeline over M micro-batches.
"""


class PipeInstruction:

    def __init__(self, **kwargs):
        self.name = self.__class__.__name__
        self.kwargs = kwargs
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __repr__(self):
        args = ", ".join(f"{k}={v}" for k, v in self.kwargs.items())
        return f"{self.name}({args})"

    def __eq__(self, other):
        return type(self) is type(other) and self.kwargs == other.kwargs


class OptimizerStep(PipeInstruction):
    pass


class ReduceGrads(PipeInstruction):
    pass


class ReduceTiedGrads(PipeInstruction):
    pass


class BufferOpInstruction(PipeInstruction):

    def __init__(self, buffer_id, **kwargs):
        super().__init__(buffer_id=buffer_id, **kwargs)


class LoadMicroBatch(BufferOpInstruction):
    pass


class ForwardPass(BufferOpInstruction):
    pass


class BackwardPass(BufferOpInstruction):
    pass


class SendActivation(BufferOpInstruction):
    pass


class RecvActivation(BufferOpInstruction):
    pass


class SendGrad(BufferOpInstruction):
    pass


class RecvGrad(BufferOpInstruction):
    pass


class PipeSchedule:

    def __init__(self, micro_batches, stages, stage_id):
        self.micro_batches = micro_batches
        self.stages = stages
        self.stage_id = stage_id
        self.prev_stage = stage_id - 1
        self.next_stage = stage_id + 1

    def steps(self):
        raise NotImplementedError

    def num_pipe_buffers(self):
        return self.micro_batches

    def _valid_micro_batch(self, mb):
        return 0 <= mb < self.micro_batches

    def _valid_stage(self, s):
        return 0 <= s < self.stages

    @property
    def is_first_stage(self):
        return self.stage_id == 0

    @property
    def is_last_stage(self):
        return self.stage_id == self.stages - 1

    def _buffer_idx(self, mb):
        return mb % self.num_pipe_buffers()

    def __iter__(self):
        self.it = None
        return self

    def __next__(self):
        if self.it is None:
            self.it = self.steps()
        return next(self.it)


class InferenceSchedule(PipeSchedule):

    def steps(self):
        for mb in range(self.micro_batches):
            cmds = []
            buf = self._buffer_idx(mb)
            if self.is_first_stage or self.is_last_stage:
                cmds.append(LoadMicroBatch(buf))
            if not self.is_first_stage:
                cmds.append(RecvActivation(buf))
            cmds.append(ForwardPass(buf))
            if not self.is_last_stage:
                cmds.append(SendActivation(buf))
            yield cmds

    def num_pipe_buffers(self):
        return 2


class TrainSchedule(PipeSchedule):

    def _forward_cmds(self, mb):
        buf = self._buffer_idx(mb)
        cmds = []
        if self.is_first_stage or self.is_last_stage:
            cmds.append(LoadMicroBatch(buf))
        if self._valid_stage(self.prev_stage):
            cmds.append(RecvActivation(buf))
        cmds.append(ForwardPass(buf))
        if self._valid_stage(self.next_stage):
            cmds.append(SendActivation(buf))
        return cmds

    def _backward_cmds(self, mb):
        buf = self._buffer_idx(mb)
        cmds = []
        if self._valid_stage(self.next_stage):
            cmds.append(RecvGrad(buf))
        cmds.append(BackwardPass(buf))
        if self._valid_stage(self.prev_stage):
            cmds.append(SendGrad(buf))
        return cmds

    def steps(self):
        M = self.micro_batches
        warmup = min(self.stages - self.stage_id - 1, M)
        fwd = bwd = 0
        plan = []
        for _ in range(warmup):
            plan.append(self._forward_cmds(fwd))
            fwd += 1
        while fwd < M:
            plan.append(self._forward_cmds(fwd))
            fwd += 1
            plan.append(self._backward_cmds(bwd))
            bwd += 1
        while bwd < M:
            plan.append(self._backward_cmds(bwd))
            bwd += 1
        # model step at the end of the batch, on every stage
        plan.append([ReduceTiedGrads(), ReduceGrads(), OptimizerStep()])
        yield from plan

    def num_pipe_buffers(self):
        return max(2, min(self.stages - self.stage_id, self.micro_batches))


class DataParallelSchedule(PipeSchedule):
    """Plain DP with gradient accumulation expressed as instructions (single stage)."""

    def steps(self):
        for mb in range(self.micro_batches):
            cmds = [LoadMicroBatch(0), ForwardPass(0), BackwardPass(0)]
            if mb == self.micro_batches - 1:
                cmds += [ReduceGrads(), OptimizerStep()]
            yield cmds

    def num_pipe_buffers(self):
        return 1
