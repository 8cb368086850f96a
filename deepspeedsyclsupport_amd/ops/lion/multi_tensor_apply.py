"""Chunked multi-tensor launcher (reference `ops/lion/multi_tensor_apply.py`): calls `op(chunk_size, noop_flag,
tensor_lists, *args)`. The gfx950 multi-tensor kernels (`csrc/optim/*.hip`) take whole tensor lists and chunk on the
device, so the chunk size is passed through unchanged."""


class MultiTensorApply:

    def __init__(self, chunk_size):
        self.chunk_size = chunk_size

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)
