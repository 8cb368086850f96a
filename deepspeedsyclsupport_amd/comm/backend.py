"""Communication backend base (reference `comm/backend.py`): what a backend object reports about itself. The one
real backend here is torch.distributed (RCCL on device tensors, gloo on host tensors), reached through the module
functions of `comm/comm.py`; backend objects exist for code that holds one."""


class Backend:

    def __init__(self, name="backend", rank=0, size=1):
        self.name = name
        self.world_group = None
        self.world_size = size
        self.world_rank = rank
        self.process_groups = []
        self.initialized = False

    def is_initialized(self):
        return self.initialized

    def new_group(self):
        raise NotImplementedError("create groups with comm.new_group")

    def init_process_group(self):
        self.initialized = True
