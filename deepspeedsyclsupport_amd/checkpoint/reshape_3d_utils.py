"""3-D (pipeline, tensor, data parallel) description of a checkpoint folder and its contraction to a smaller topology
(reference `checkpoint/reshape_3d_utils.py:17-118`)."""
from . import constants as CK
from .reshape_meg_2d import meg_2d_parallel_map, reshape_meg_2d_parallel
from .reshape_utils import get_files, get_files_with_prefix, get_zero_files, partition_data

PP_DIM, TP_DIM, DP_DIM = "PP", "TP", "DP"


class model_3d_desc:

    def __init__(self, pp_degree=1, tp_degree=1, dp_degree=1):
        self.pp_degree, self.tp_degree, self.dp_degree = pp_degree, tp_degree, dp_degree

    def get_desc(self):
        return f"{PP_DIM},{TP_DIM},{DP_DIM} = ({self.pp_degree}, {self.tp_degree}, {self.dp_degree})"

    def world_size(self):
        return self.pp_degree * self.tp_degree * self.dp_degree

    def is_valid(self, pp_index, tp_index, dp_index):
        errs = [f"{name} indexing error: index {i} >= degree {deg}"
                for i, deg, name in ((pp_index, self.pp_degree, PP_DIM), (tp_index, self.tp_degree, TP_DIM),
                                     (dp_index, self.dp_degree, DP_DIM)) if i >= deg]
        return not errs, errs

    def can_reshape(self, target):
        errs = [f"Expansion reshape not supported - {name}: {mine} ---> {theirs}"
                for mine, theirs, name in ((self.pp_degree, target.pp_degree, PP_DIM),
                                           (self.tp_degree, target.tp_degree, TP_DIM),
                                           (self.dp_degree, target.dp_degree, DP_DIM)) if theirs > mine]
        return not errs, errs

    def reshape(self, target, verbose=False):
        """One 2-D map per TARGET data-parallel rank: cell (pp, tp) -> source zero-file indices it merges. A source
        file index is model_rank + dp_index * (pp * tp)."""
        ok, errs = self.can_reshape(target)
        if not ok:
            raise ValueError(",".join(errs))
        two_d = reshape_meg_2d_parallel(self.pp_degree, self.tp_degree, target.pp_degree, target.tp_degree, verbose)
        return unflatten_dp_dimension(flatten_dp_dimension(two_d, self.pp_degree * self.tp_degree, self.dp_degree),
                                      target.dp_degree)


def flatten_dp_dimension(meg_2d_map, src_2d_size, dp_degree):
    out = meg_2d_parallel_map(meg_2d_map.pp_degree, meg_2d_map.tp_degree)
    for i in range(meg_2d_map.pp_degree):
        for j in range(meg_2d_map.tp_degree):
            for idx in meg_2d_map.get_data(i, j):
                out.add_data(i, j, [idx + d * src_2d_size for d in range(dp_degree)])
    return out


def unflatten_dp_dimension(meg_2d_map, dp_degree):
    maps = [meg_2d_parallel_map(meg_2d_map.pp_degree, meg_2d_map.tp_degree) for _ in range(dp_degree)]
    for i in range(meg_2d_map.pp_degree):
        for j in range(meg_2d_map.tp_degree):
            for m, part in zip(maps, partition_data(meg_2d_map.get_data(i, j), dp_degree)):
                m.add_data(i, j, part)
    return maps


def get_model_3d_descriptor(dir):
    """Infer (pp, tp, dp) from the files of a checkpoint folder: pipeline checkpoints have `layer_XX-model_YY` files
    (YY = tensor-parallel rank), others one `mp_rank_XX` file per tensor-parallel rank."""
    files = get_files(dir)
    zero = get_zero_files(dir)
    model_files = [f for f in get_files_with_prefix(files, CK.MODEL_FILE_PREFIX) if f.endswith(CK.MODEL_FILE_SUFFIX)]
    first_layer = get_files_with_prefix(files, f"{CK.LAYER_FILE_PREFIX}01")
    if first_layer:
        tp = len(first_layer)
        pp = max(len(model_files) // tp, 1)
    else:
        tp, pp = max(len(model_files), 1), 1
    return model_3d_desc(pp, tp, max(1, len(zero) // (pp * tp)))
