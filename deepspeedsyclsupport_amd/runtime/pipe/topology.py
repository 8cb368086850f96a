"""Process topologies and the pipeline grid (API of the reference `runtime/pipe/topology.py:12-456`:
ProcessTopology / PipeDataParallelTopology / PipeModelDataParallelTopology / PipelineParallelGrid).

A topology is a mixed-radix numbering of ranks over named axes, the LAST axis varying fastest. Everything here is
plain radix arithmetic — coordinates are digits, a communicator along one axis is the set of ranks that differ only
in that digit — rather than enumerating and searching a coordinate table.

MI355X placement: with 'model' (TP) innermost the tensor-parallel peers are adjacent ranks, and with 'pipe' outermost
neighbouring pipeline stages are adjacent rank blocks; on one node every pair of GPUs has its own xGMI link, so the
choice mainly keeps TP groups inside one node when jobs span nodes.
"""
from collections import namedtuple

from ... import comm as dist


class ProcessTopology:
    """Ranks laid out on a grid with named axes (row-major: the last axis has stride 1)."""

    def __init__(self, axes, dims):
        if len(axes) != len(dims) or any(d <= 0 for d in dims):
            raise ValueError(f"bad topology axes={axes} dims={dims}")
        self.axes = list(axes)
        self.dims = [int(d) for d in dims]
        self.ProcessCoord = namedtuple("ProcessCoord", self.axes)
        self._stride = []
        s = 1
        for d in reversed(self.dims):
            self._stride.insert(0, s)
            s *= d
        self._size = s

    # ---- coordinates <-> ranks
    def _rank_of(self, digits):
        return sum(d * st for d, st in zip(digits, self._stride))

    def _digits_of(self, rank):
        return [(rank // st) % d for st, d in zip(self._stride, self.dims)]

    def get_rank(self, **coord_kwargs):
        if set(coord_kwargs) != set(self.axes):
            raise ValueError("get_rank() needs every axis; use filter_match() for partial coordinates")
        return self._rank_of([coord_kwargs[a] for a in self.axes])

    def get_coord(self, rank):
        if not 0 <= rank < self._size:
            raise ValueError(f"rank {rank} not found in topology.")
        return self.ProcessCoord(*self._digits_of(rank))

    @property
    def mapping(self):
        return {self.get_coord(r): r for r in range(self._size)}

    # ---- queries
    def get_axis_names(self):
        return list(self.axes)

    def get_dim(self, axis):
        return self.dims[self.axes.index(axis)] if axis in self.axes else 0

    def world_size(self):
        return self._size

    def get_rank_repr(self, rank, omit_axes=("data", "pipe"), inner_sep="_", outer_sep="-"):
        coord = self.get_coord(rank)
        return outer_sep.join(f"{a}{inner_sep}{getattr(coord, a):02d}" for a in self.axes if a not in omit_axes)

    def filter_match(self, **filter_kwargs):
        """Ranks whose coordinates match every given axis value, ascending."""
        idx = {self.axes.index(a): v for a, v in filter_kwargs.items()}
        return [r for r in range(self._size) if all(self._digits_of(r)[i] == v for i, v in idx.items())]

    def get_axis_list(self, axis, idx):
        return self.filter_match(**{axis: idx})

    def get_axis_comm_lists(self, axis):
        """One list per fixed setting of the other axes: the ranks along `axis` (communicators for that axis)."""
        if axis not in self.axes:
            return []
        k = self.axes.index(axis)
        out = []
        for r in range(self._size):
            if self._digits_of(r)[k] == 0:  # first member of each line
                out.append([r + i * self._stride[k] for i in range(self.dims[k])])
        return out

    def __str__(self):
        return str(self.mapping)


class PipeDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_dp):
        super().__init__(axes=["pipe", "data"], dims=[num_pp, num_dp])


class PipeModelDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


def _default_split(world):
    """pipe x data factorisation used when no topology is given: alternate the prime factors between the two."""
    pp = dp = 1
    n, f, turn = world, 2, 0
    while n > 1:
        while n % f == 0:
            if turn % 2 == 0:
                pp *= f
            else:
                dp *= f
            turn += 1
            n //= f
        f += 1
    return pp, dp


class PipelineParallelGrid:
    """Every process group a pipeline (+data, +model) job needs, plus the mpu-style query interface."""

    def __init__(self, topology=None, process_group=None):
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if topology is None:
            pp, dp = _default_split(self.world_size)
            topology = PipeDataParallelTopology(num_pp=pp, num_dp=dp)
        self._topo = topology
        if self._topo.world_size() != self.world_size:
            raise AssertionError("Invalid Grid")
        self.data_parallel_size = max(self._topo.get_dim("data"), 1)
        self.pipe_parallel_size = max(self._topo.get_dim("pipe"), 1)
        self.model_parallel_size = max(self._topo.get_dim("model"), 1)
        self.slice_parallel_size = self.model_parallel_size
        me = self._topo.get_coord(self.global_rank)
        self.stage_id = me.pipe
        self.data_parallel_id = me.data
        self.is_first_stage = self.stage_id == 0
        self.is_last_stage = self.stage_id == self.pipe_parallel_size - 1

        # groups are created collectively: every rank walks the same lists in the same order
        def make(lists):
            mine = None
            for ranks in lists:
                g = dist.new_group(ranks=ranks)
                if self.global_rank in ranks:
                    mine = (ranks, g)
            return mine or ([self.global_rank], None)

        # "model" replica = all ranks holding one data-parallel copy (every pipe stage and model slice)
        replicas = [self._topo.filter_match(data=d) for d in range(self.data_parallel_size)]
        ranks, self.ds_model_proc_group = make(replicas)
        self.ds_model_world_size = len(ranks)
        self.ds_model_rank = ranks.index(self.global_rank)
        self.dp_group, self.dp_proc_group = make(self._topo.get_axis_comm_lists("data"))
        self.pp_group, self.pp_proc_group = make(self._topo.get_axis_comm_lists("pipe"))
        if self.model_parallel_size > 1:
            mp_lists = self._topo.get_axis_comm_lists("model")
        else:
            mp_lists = [[r] for r in range(self.world_size)]
        self.mp_group, self.model_parallel_group = make(mp_lists)
        self.slice_group, self.slice_proc_group = self.mp_group, self.model_parallel_group
        self.p2p_groups = self._build_p2p_groups()

    def _build_p2p_groups(self):
        """[rank, next stage's rank] for every rank (the ring of its pipeline)."""
        nxt = {}
        for line in self._topo.get_axis_comm_lists("pipe"):
            for i, r in enumerate(line):
                nxt[r] = line[(i + 1) % len(line)]
        return [[r, nxt.get(r, r)] for r in range(self.world_size)]

    def get_stage_id(self):
        return self.stage_id

    def get_data_parallel_id(self):
        return self.data_parallel_id

    def stage_to_global(self, stage_id, **kwargs):
        coord = self._topo.get_coord(self.global_rank)._replace(pipe=stage_id, **kwargs)
        return self._topo.get_rank(**coord._asdict())

    def topology(self):
        return self._topo

    # ---- mpu interface
    def get_global_rank(self):
        return self.global_rank

    def get_pipe_parallel_rank(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self):
        return self.pp_proc_group

    def get_data_parallel_rank(self):
        return self.data_parallel_id

    def get_data_parallel_world_size(self):
        return self.data_parallel_size

    def get_data_parallel_group(self):
        return self.dp_proc_group

    # "model parallel" for the engine = everything that is not data parallel (pipe stages x tensor slices), as in the
    # reference grid (`runtime/pipe/topology.py:436-443`): checkpoint file names and mp_world_size are built on it
    def get_model_parallel_rank(self):
        return self.ds_model_rank

    def get_model_parallel_world_size(self):
        return self.ds_model_world_size

    def get_model_parallel_group(self):
        return self.ds_model_proc_group

    def get_slice_parallel_rank(self):
        return self._topo.get_coord(self.global_rank).model if "model" in self._topo.get_axis_names() else 0

    def get_slice_parallel_world_size(self):
        return self.slice_parallel_size

    def get_slice_parallel_group(self):
        return self.slice_proc_group
