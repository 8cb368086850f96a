"""Offline data analysis for curriculum learning (reference `runtime/data_pipeline/data_sampling/data_analyzer.py:20-418`).

Map: every (worker, thread) walks its contiguous slice of the dataset in batches and applies each metric function:
  * `single_value_per_sample`      -> one integer difficulty per sample (e.g. sequence length, vocab rarity);
  * `accumulate_value_over_samples`-> an integer vector summed over all samples (e.g. token histograms).
Results go to `<save_path>/<metric>/worker<w>_thread<t>/` as an MMIDIDX dataset (`<metric>_sample_to_metric`,
`<metric>_metric_value`) plus the raw (sample, value) pairs as .npy (allow_pickle never needed).

Reduce: merges all map outputs into the files the curriculum sampler reads, with the reference's names:
  `<metric>_sample_to_metric`   value of every sample, in sample order
  `<metric>_index_to_sample`    one item per distinct value (ascending): the samples having it
  `<metric>_index_to_metric`    that value
  `<metric>_index_to_sample_percentile_merged`  the same lists merged into ~100 percentile buckets
  `<metric>_metric_value`       the accumulated vector (accumulate type)
Instead of the reference's per-value CSV spill files and per-value merge loops, the reduce is one stable numpy sort
of the (value, sample) pairs followed by a split at the value boundaries.
"""
import os

import numpy as np
import torch
from torch.utils.data import BatchSampler, DataLoader, SequentialSampler, Subset

from ....utils.logging import logger
from .indexed_dataset import (MMapIndexedDataset, close_mmap_dataset_builder, create_mmap_dataset_builder,
                              find_fit_int_dtype)

SINGLE = "single_value_per_sample"
ACCUM = "accumulate_value_over_samples"


def split_index(start_idx, end_idx, num_partitions):
    """Contiguous, balanced split of [start_idx, end_idx) (reference `data_sampling/utils.py:34`)."""
    edges = np.linspace(start_idx, end_idx, num_partitions + 1).astype(np.int64)
    return [(int(edges[i]), int(edges[i + 1])) for i in range(num_partitions)]


def split_dataset(dataset, num_workers, worker_id, num_threads):
    worker_splits = split_index(0, len(dataset), num_workers)
    s, e = worker_splits[worker_id]
    return worker_splits, split_index(s, e, num_threads)


class DataAnalyzer:

    def __init__(self, dataset, num_workers=1, worker_id=0, num_threads=1, num_threads_reduce=1, specific_threads=(),
                 batch_size=1, metric_names=(), metric_functions=(), metric_types=(), metric_dtypes=(),
                 save_path="./", collate_fn=None, custom_map_init=None, custom_map_update=None,
                 custom_map_finalize=None, custom_reduce=None):
        self.dataset = dataset
        self.num_workers, self.worker_id = num_workers, worker_id
        self.num_threads, self.num_threads_reduce = num_threads, num_threads_reduce
        self.specific_threads = list(specific_threads)
        self.batch_size = batch_size
        self.metric_names, self.metric_functions = list(metric_names), list(metric_functions)
        self.metric_types, self.metric_dtypes = list(metric_types), list(metric_dtypes)
        for t in self.metric_dtypes:
            assert not np.issubdtype(np.dtype(t), np.floating), "metric values must be integers (scale them)"
        self.save_path = save_path
        self.collate_fn = collate_fn
        self.custom_map_init, self.custom_map_update = custom_map_init, custom_map_update
        self.custom_map_finalize, self.custom_reduce = custom_map_finalize, custom_reduce

    # ------------------------------------------------------------------------------------------ map
    def _dir(self, name, w, t):
        d = os.path.join(self.save_path, name, f"worker{w}_thread{t}")
        os.makedirs(d, exist_ok=True)
        return d

    def run_map_helper(self, thread_id):
        start, end = self.thread_splits[thread_id]
        subset = Subset(self.dataset, list(range(start, end)))
        loader = DataLoader(subset, batch_sampler=BatchSampler(SequentialSampler(subset), self.batch_size, False),
                            num_workers=0, collate_fn=self.collate_fn)
        state = [{"idx": [], "val": [], "acc": None} for _ in self.metric_names]
        if self.custom_map_init is not None:
            state = self.custom_map_init(thread_id, self.metric_names, self.metric_types, self.metric_dtypes,
                                         self.save_path, self.worker_id)
        pos = start
        for batch in loader:
            if self.custom_map_update is not None:
                self.custom_map_update(batch, self.metric_types, self.metric_functions, state)
                continue
            n = None
            for m, (mtype, fn) in enumerate(zip(self.metric_types, self.metric_functions)):
                vals = fn(batch)
                vals = vals.detach().cpu() if torch.is_tensor(vals) else torch.as_tensor(vals)
                if mtype == SINGLE:
                    vals = vals.reshape(-1).to(torch.int64).numpy()
                    n = vals.size
                    state[m]["idx"].append(np.arange(pos, pos + n, dtype=np.int64))
                    state[m]["val"].append(vals)
                elif mtype == ACCUM:
                    acc = state[m]["acc"]
                    state[m]["acc"] = vals.to(torch.int64) if acc is None else acc + vals.to(torch.int64)
                else:
                    raise ValueError(f"unknown metric type {mtype}")
            pos += n if n is not None else self.batch_size
        if self.custom_map_finalize is not None:
            self.custom_map_finalize(self.metric_types, self.metric_dtypes, state)
            return
        for m, name in enumerate(self.metric_names):
            d = self._dir(name, self.worker_id, thread_id)
            if self.metric_types[m] == SINGLE:
                idx = np.concatenate(state[m]["idx"]) if state[m]["idx"] else np.zeros(0, np.int64)
                val = np.concatenate(state[m]["val"]) if state[m]["val"] else np.zeros(0, np.int64)
                np.save(os.path.join(d, f"{name}_pairs_idx.npy"), idx)
                np.save(os.path.join(d, f"{name}_pairs_val.npy"), val)
                b = create_mmap_dataset_builder(os.path.join(d, f"{name}_sample_to_metric"), self.metric_dtypes[m])
                b.add_items_numpy(val, np.ones(val.size, dtype=np.int64))
                close_mmap_dataset_builder(b, os.path.join(d, f"{name}_sample_to_metric"))
            elif state[m]["acc"] is not None:
                fname = os.path.join(d, f"{name}_metric_value")
                b = create_mmap_dataset_builder(fname, self.metric_dtypes[m])
                b.add_item(state[m]["acc"].reshape(-1))
                close_mmap_dataset_builder(b, fname)
        logger.info(f"data analyzer: worker {self.worker_id} thread {thread_id} mapped samples [{start}, {end})")

    def run_map(self):
        self.worker_splits, self.thread_splits = split_dataset(self.dataset, self.num_workers, self.worker_id,
                                                               self.num_threads)
        threads = self.specific_threads or list(range(self.num_threads))
        if self.num_threads > 1:
            import multiprocessing as mp
            ctx = mp.get_context("fork")
            procs = [ctx.Process(target=self.run_map_helper, args=(t, )) for t in threads]
            for p in procs:
                p.start()
            for p in procs:
                p.join()
                assert p.exitcode == 0, f"map thread failed with exit code {p.exitcode}"
        else:
            self.run_map_helper(threads[0] if threads else 0)

    # ------------------------------------------------------------------------------------------ reduce
    def merge_map_results(self, dataset, metric_names, metric_types, save_path, num_workers, num_threads,
                          num_threads_reduce):
        total = len(dataset)
        sample_dtype = find_fit_int_dtype(0, max(total - 1, 0))
        for name, mtype in zip(metric_names, metric_types):
            base = os.path.join(save_path, name)
            if mtype == SINGLE:
                idx_parts, val_parts = [], []
                for w in range(num_workers):
                    for t in range(num_threads):
                        d = os.path.join(base, f"worker{w}_thread{t}")
                        idx_parts.append(np.load(os.path.join(d, f"{name}_pairs_idx.npy")))
                        val_parts.append(np.load(os.path.join(d, f"{name}_pairs_val.npy")))
                idx, val = np.concatenate(idx_parts), np.concatenate(val_parts)
                assert idx.size == total, f"map results cover {idx.size} of {total} samples (a map worker failed?)"
                vdtype = find_fit_int_dtype(int(val.min()), int(val.max())) if val.size else np.int64
                by_sample = np.empty(total, dtype=np.int64)
                by_sample[idx] = val
                f = os.path.join(base, f"{name}_sample_to_metric")
                b = create_mmap_dataset_builder(f, vdtype)
                b.add_items_numpy(by_sample, np.ones(total, dtype=np.int64))
                close_mmap_dataset_builder(b, f)
                order = np.lexsort((idx, val))  # by value, ties by sample index
                sv, si = val[order], idx[order]
                uniq, starts, counts = np.unique(sv, return_index=True, return_counts=True)
                f_is = os.path.join(base, f"{name}_index_to_sample")
                f_im = os.path.join(base, f"{name}_index_to_metric")
                bi = create_mmap_dataset_builder(f_is, sample_dtype)
                bi.add_items_numpy(si, counts)
                close_mmap_dataset_builder(bi, f_is)
                bm = create_mmap_dataset_builder(f_im, vdtype)
                bm.add_items_numpy(uniq, np.ones(uniq.size, dtype=np.int64))
                close_mmap_dataset_builder(bm, f_im)
                # ~100 percentile buckets of whole value groups
                step = max(1, uniq.size // 100)
                merged_sizes = [int(counts[i:i + step].sum()) for i in range(0, uniq.size, step)]
                f_pm = os.path.join(base, f"{name}_index_to_sample_percentile_merged")
                bp = create_mmap_dataset_builder(f_pm, sample_dtype)
                bp.add_items_numpy(si, merged_sizes)
                close_mmap_dataset_builder(bp, f_pm)
                cum = np.cumsum(counts)
                pct = {p: int(uniq[np.searchsorted(cum, total * p / 100.0)]) for p in range(5, 100, 5)}
                logger.info(f"metric {name}: values {int(uniq[0])}..{int(uniq[-1])}, percentiles {pct}")
            elif mtype == ACCUM:
                acc = None
                for w in range(num_workers):
                    for t in range(num_threads):
                        f = os.path.join(base, f"worker{w}_thread{t}", f"{name}_metric_value")
                        if MMapIndexedDataset.exists(f):
                            v = np.asarray(MMapIndexedDataset(f)[0], dtype=np.int64)
                            acc = v.copy() if acc is None else acc + v
                if acc is None:
                    continue
                vdtype = find_fit_int_dtype(int(acc.min()), int(acc.max()))
                f = os.path.join(base, f"{name}_metric_value")
                b = create_mmap_dataset_builder(f, vdtype)
                b.add_item_numpy(acc)
                close_mmap_dataset_builder(b, f)

    def run_reduce(self):
        fn = self.custom_reduce or self.merge_map_results
        fn(self.dataset, self.metric_names, self.metric_types, self.save_path, self.num_workers, self.num_threads,
           self.num_threads_reduce)
