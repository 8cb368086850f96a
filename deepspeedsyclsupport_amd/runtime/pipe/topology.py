"""Process topologies and the pipeline grid (reference `runtime/pipe/topology.py:12-456`).

A topology is a cartesian grid of named axes (e.g. ['pipe', 'data'] or ['pipe', 'data', 'model']); rank =
row-major index. On an 8-GPU MI355X node, putting 'model' (TP) innermost keeps tensor-parallel peers adjacent and
'pipe' outermost makes neighbouring pipeline stages adjacent rank blocks — every p2p hop and TP collective then stays
on direct xGMI links of the full mesh.
"""
from collections import namedtuple
from itertools import product as cartesian_product

from ... import comm as dist


class ProcessTopology:

    def __init__(self, axes, dims):
        self.axes = list(axes)
        self.dims = list(dims)
        self.ProcessCoord = namedtuple("ProcessCoord", axes)
        self.mapping = {}
        ranges = [range(d) for d in dims]
        for global_rank, coord in enumerate(cartesian_product(*ranges)):
            key = self.ProcessCoord(**{axis: coord[self.axes.index(axis)] for axis in self.axes})
            self.mapping[key] = global_rank

    def get_rank(self, **coord_kwargs):
        if len(coord_kwargs) != len(self.axes):
            raise ValueError("get_rank() does not support slices. Use filter_match())")
        return self.mapping[self.ProcessCoord(**coord_kwargs)]

    def get_axis_names(self):
        return self.axes

    def get_rank_repr(self, rank, omit_axes=["data", "pipe"], inner_sep="_", outer_sep="-"):
        omit = frozenset(omit_axes)
        axes = [a for a in self.get_axis_names() if a not in omit]
        names = []
        for ax in axes:
            names.append(f"{ax}{inner_sep}{self.get_coord(rank=rank)._asdict()[ax]:02d}")
        return outer_sep.join(names)

    def get_dim(self, axis):
        if axis not in self.axes:
            return 0
        return self.dims[self.axes.index(axis)]

    def get_coord(self, rank):
        for coord, idx in self.mapping.items():
            if idx == rank:
                return coord
        raise ValueError(f"rank {rank} not found in topology.")

    def get_axis_comm_lists(self, axis):
        if axis not in self.axes:
            return []
        other = [a for a in self.axes if a != axis]
        lists = []
        ranges = [range(self.get_dim(a)) for a in other]
        for coord in cartesian_product(*ranges):
            other_keys = {a: coord[other.index(a)] for a in other}
            sub = []
            for i in range(self.get_dim(axis)):
                sub.append(self.mapping[self.ProcessCoord(**other_keys, **{axis: i})])
            lists.append(sub)
        return lists

    def filter_match(self, **filter_kwargs):

        def _filter(x):
            for key, val in filter_kwargs.items():
                if getattr(x, key) != val:
                    return False
            return True

        return [self.mapping[c] for c in filter(_filter, self.mapping.keys())]

    def get_axis_list(self, axis, idx):
        axis_num = self.axes.index(axis)
        return [self.mapping[k] for k in self.mapping.keys() if k[axis_num] == idx]

    def world_size(self):
        n = 1
        for d in self.dims:
            n *= d
        return n

    def __str__(self):
        return str(self.mapping)


def _prime_factors(N):
    if N <= 0:
        raise ValueError("Values must be strictly positive.")
    primes = []
    while N != 1:
        for candidate in range(2, N + 1):
            if N % candidate == 0:
                primes.append(candidate)
                N //= candidate
                break
    return primes


class PipeDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_dp):
        super().__init__(axes=["pipe", "data"], dims=[num_pp, num_dp])


class PipeModelDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


class PipelineParallelGrid:
    """Builds every process group a pipeline(+data/+model) job needs and answers mpu-style queries."""

    def __init__(self, topology=None, process_group=None):
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if topology is not None:
            self._topo = topology
        else:
            num_pp = 1
            num_dp = 1
            for idx, prime in enumerate(_prime_factors(self.world_size)):
                if idx % 2 == 0:
                    num_pp *= prime
                else:
                    num_dp *= prime
            self._topo = PipeDataParallelTopology(num_dp=num_dp, num_pp=num_pp)
        self.data_parallel_size = max(self._topo.get_dim("data"), 1)
        self.pipe_parallel_size = max(self._topo.get_dim("pipe"), 1)
        self.model_parallel_size = max(self._topo.get_dim("model"), 1)
        self.slice_parallel_size = self.model_parallel_size
        assert self._is_grid_valid(), "Invalid Grid"
        self.stage_id = self.get_stage_id()
        self.data_parallel_id = self.get_data_parallel_id()

        self.ds_model_proc_group = None
        self.ds_model_rank = -1
        for dp in range(self.data_parallel_size):
            ranks = sorted(self._topo.get_axis_list(axis="data", idx=dp))
            g = dist.new_group(ranks=ranks)
            if self.global_rank in ranks:
                self.ds_model_proc_group = g
                self.ds_model_world_size = len(ranks)
                self.ds_model_rank = ranks.index(self.global_rank)
        self.dp_group = []
        self.dp_proc_group = None
        for g_ranks in self._topo.get_axis_comm_lists("data"):
            proc = dist.new_group(ranks=g_ranks)
            if self.global_rank in g_ranks:
                self.dp_group = g_ranks
                self.dp_proc_group = proc
        self.is_first_stage = self.stage_id == 0
        self.is_last_stage = self.stage_id == self.pipe_parallel_size - 1
        self.p2p_groups = self._build_p2p_groups()
        self.pp_group = []
        self.pp_proc_group = None
        for ranks in self._topo.get_axis_comm_lists("pipe"):
            proc = dist.new_group(ranks=ranks)
            if self.global_rank in ranks:
                self.pp_group = ranks
                self.pp_proc_group = proc
        self.slice_group = None
        self.slice_proc_group = None
        self.mp_group = []
        self.model_parallel_group = None
        if self.model_parallel_size > 1:
            for ranks in self._topo.get_axis_comm_lists("model"):
                proc = dist.new_group(ranks=ranks)
                if self.global_rank in ranks:
                    self.slice_group = ranks
                    self.slice_proc_group = proc
                    self.model_parallel_group = proc
                    self.mp_group = ranks
        else:
            for r in range(self.world_size):
                g = dist.new_group(ranks=[r])
                if r == self.global_rank:
                    self.slice_group = [r]
                    self.slice_proc_group = g
                    self.model_parallel_group = g
                    self.mp_group = [r]

    def get_stage_id(self):
        return self._topo.get_coord(rank=self.global_rank).pipe

    def get_data_parallel_id(self):
        return self._topo.get_coord(rank=self.global_rank).data

    def _build_p2p_groups(self):
        comm_lists = self._topo.get_axis_comm_lists("pipe")
        p2p_lists = []
        for rank in range(self.world_size):
            for l in comm_lists:
                assert len(l) == self.pipe_parallel_size
                if rank in l:
                    idx = l.index(rank)
                    buddy_rank = l[(idx + 1) % self.pipe_parallel_size]
                    p2p_lists.append([rank, buddy_rank])
                    break
        assert len(p2p_lists) == self.world_size
        return p2p_lists

    def _is_grid_valid(self):
        ranks = 1
        for ax in self._topo.get_axis_names():
            ranks *= self._topo.get_dim(ax)
        return ranks == dist.get_world_size()

    def stage_to_global(self, stage_id, **kwargs):
        me = self._topo.get_coord(self.global_rank)
        transform = me._replace(pipe=stage_id, **kwargs)._asdict()
        return self._topo.get_rank(**transform)

    def topology(self):
        return self._topo

    # mpu interface
    def get_global_rank(self):
        return self.global_rank

    def get_pipe_parallel_rank(self):
        return self.get_stage_id()

    def get_pipe_parallel_world_size(self):
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self):
        return self.pp_proc_group

    def get_data_parallel_rank(self):
        return self.get_data_parallel_id()

    def get_data_parallel_world_size(self):
        return self.data_parallel_size

    def get_data_parallel_group(self):
        return self.dp_proc_group

    def get_model_parallel_rank(self):
        return self.ds_model_rank if self.model_parallel_size == 1 else \
            self._topo.get_coord(rank=self.global_rank).model

    def get_model_parallel_world_size(self):
        return self.model_parallel_size

    def get_model_parallel_group(self):
        return self.model_parallel_group

    def get_slice_parallel_rank(self):
        return self.get_model_parallel_rank() if "model" in self._topo.get_axis_names() else 0

    def get_slice_parallel_world_size(self):
        return self.slice_parallel_size

    def get_slice_parallel_group(self):
        return self.slice_proc_group
