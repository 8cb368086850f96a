"""Pipeline x tensor parallel rank maps and their contraction to a smaller grid (reference
`checkpoint/reshape_meg_2d.py:9-228`).

A source grid of `pp x tp` model-parallel ranks is numbered row-major (rank = pp_index * tp + tp_index, Megatron's
order). Shrinking it assigns to every cell of the target grid the source ranks whose shards it must merge: tensor
parallel neighbours first (contiguous runs of a row), then pipeline neighbours (contiguous runs of a column). Kept as
an integer array of rank lists instead of a string-keyed dict.
"""
import numpy as np

from .reshape_utils import partition_data


class meg_2d_parallel_map:
    """cell (pp_index, tp_index) -> list of source rank indices."""

    def __init__(self, pp_degree, tp_degree):
        self.pp_degree, self.tp_degree = int(pp_degree), int(tp_degree)
        self.cells = np.empty((self.pp_degree, self.tp_degree), dtype=object)
        for i in range(self.pp_degree):
            for j in range(self.tp_degree):
                self.cells[i, j] = []

    def simple_init(self):
        for i in range(self.pp_degree):
            for j in range(self.tp_degree):
                self.cells[i, j] = [i * self.tp_degree + j]

    def _check(self, pp_index, tp_index):
        if pp_index is not None and not 0 <= pp_index < self.pp_degree:
            raise IndexError(f"pp index {pp_index} outside degree {self.pp_degree}")
        if tp_index is not None and not 0 <= tp_index < self.tp_degree:
            raise IndexError(f"tp index {tp_index} outside degree {self.tp_degree}")

    def add_data(self, pp_index, tp_index, data):
        self._check(pp_index, tp_index)
        if not isinstance(data, list):
            raise TypeError("data must be a list of rank indices")
        self.cells[pp_index, tp_index] = self.cells[pp_index, tp_index] + data

    def get_data(self, pp_index=None, tp_index=None):
        """Ranks of one cell, one row (tp_index None), one column (pp_index None) or the whole grid, row-major."""
        self._check(pp_index, tp_index)
        rows = range(self.pp_degree) if pp_index is None else (pp_index, )
        cols = range(self.tp_degree) if tp_index is None else (tp_index, )
        return [r for i in rows for j in cols for r in self.cells[i, j]]

    def print_data(self, tag):
        print(tag)
        for i in range(self.pp_degree):
            for j in range(self.tp_degree):
                print(f"{i},{j} = {self.cells[i, j]}")


def _reshape_tp_dimension(old, new_tp_degree):
    new = meg_2d_parallel_map(old.pp_degree, new_tp_degree)
    for i in range(old.pp_degree):
        for j, part in enumerate(partition_data(old.get_data(pp_index=i), new_tp_degree)):
            new.add_data(i, j, part)
    return new


def _reshape_pp_dimension(old, new_pp_degree):
    new = meg_2d_parallel_map(new_pp_degree, old.tp_degree)
    for j in range(old.tp_degree):
        for i, part in enumerate(partition_data(old.get_data(tp_index=j), new_pp_degree)):
            new.add_data(i, j, part)
    return new


def reshape_meg_2d_parallel(old_pp_degree, old_tp_degree, new_pp_degree, new_tp_degree, verbose=False):
    if new_pp_degree > old_pp_degree or new_tp_degree > old_tp_degree:
        raise ValueError("only contraction of the model-parallel grid is supported")
    m = meg_2d_parallel_map(old_pp_degree, old_tp_degree)
    m.simple_init()
    if verbose:
        m.print_data("original_2d_map:")
    if new_tp_degree != old_tp_degree:
        m = _reshape_tp_dimension(m, new_tp_degree)
    if new_pp_degree != old_pp_degree:
        m = _reshape_pp_dimension(m, new_pp_degree)
    if verbose:
        m.print_data("final_2d_map:")
    return m


def get_mpu_ranks(tp_size=1, pp_size=1, dp_size=1, virtual_pp_size=None):
    """Rank groups of Megatron's rank order, rank = (pp_index * dp + dp_index) * tp + tp_index. Returns
    (tensor-parallel groups, model-replica groups, data-parallel groups): the middle list has one entry per
    data-parallel index holding every rank of that model replica (pipeline-major, then tensor), which is what the
    reference's function of this name returns under the label "PP"."""
    grid = np.arange(tp_size * pp_size * dp_size).reshape(pp_size, dp_size, tp_size)
    tp_groups = [grid[p, d, :].tolist() for p in range(pp_size) for d in range(dp_size)]
    dp_groups = [grid[p, :, t].tolist() for p in range(pp_size) for t in range(tp_size)]
    replica_groups = [grid[:, d, :].reshape(-1).tolist() for d in range(dp_size)]
    return tp_groups, replica_groups, dp_groups
