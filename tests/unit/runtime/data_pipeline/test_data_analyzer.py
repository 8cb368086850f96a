"""Indexed dataset format + DataAnalyzer map/reduce + curriculum sampler fed by the analyzer's files
(reference `tests/unit/runtime/test_data_efficiency.py`, `data_sampling/{indexed_dataset,data_analyzer}.py`)."""
import struct

import numpy as np
import pytest
import torch

from deepspeedsyclsupport_amd.runtime.data_pipeline.data_sampling import (DataAnalyzer, DeepSpeedDataSampler,
                                                                          MMapIndexedDataset,
                                                                          MMapIndexedDatasetBuilder)


def test_mmap_roundtrip_and_format(tmp_path):
    prefix = str(tmp_path / "ds")
    b = MMapIndexedDatasetBuilder(prefix + ".bin", dtype=np.uint16)
    items = [np.arange(n, dtype=np.uint16) * 3 for n in (5, 0, 17, 1)]
    for i, it in enumerate(items):
        b.add_item(torch.from_numpy(it.astype(np.int64)))
        if i == 1:
            b.end_document()
    b.end_document()
    b.finalize(prefix + ".idx")
    raw = open(prefix + ".idx", "rb").read()
    assert raw[:9] == b"MMIDIDX\x00\x00" and struct.unpack("<Q", raw[9:17])[0] == 1 and raw[17] == 8  # uint16 code
    ds = MMapIndexedDataset(prefix)
    assert len(ds) == 4 and list(ds.sizes) == [5, 0, 17, 1] and list(ds.doc_idx) == [0, 2, 4]
    for got, want in zip(ds[0:4], items):
        np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ds.get(2, offset=3, length=4), items[2][3:7])
    # merge
    p2 = str(tmp_path / "ds2")
    b2 = MMapIndexedDatasetBuilder(p2 + ".bin", dtype=np.uint16)
    b2.merge_file_(prefix)
    b2.merge_file_(prefix)
    b2.finalize(p2 + ".idx")
    d2 = MMapIndexedDataset(p2)
    assert len(d2) == 8
    np.testing.assert_array_equal(d2[6], items[2])


class _Seqs(torch.utils.data.Dataset):

    def __init__(self, n):
        g = np.random.default_rng(0)
        self.lens = g.integers(1, 40, size=n)

    def __len__(self):
        return len(self.lens)

    def __getitem__(self, i):
        x = torch.zeros(40, dtype=torch.long)
        x[:self.lens[i]] = 1 + (torch.arange(int(self.lens[i])) % 7)
        return x


@pytest.mark.parametrize("workers,threads", [(1, 1), (2, 2)])
def test_data_analyzer_map_reduce(tmp_path, workers, threads):
    ds = _Seqs(103)
    kw = dict(batch_size=8, metric_names=["seqlen", "vocab"],
              metric_functions=[lambda b: (b != 0).sum(1), lambda b: torch.bincount(b.reshape(-1), minlength=8)],
              metric_types=["single_value_per_sample", "accumulate_value_over_samples"],
              metric_dtypes=[np.int64, np.int64], save_path=str(tmp_path))
    for w in range(workers):
        DataAnalyzer(ds, num_workers=workers, worker_id=w, num_threads=threads, **kw).run_map()
    DataAnalyzer(ds, num_workers=workers, num_threads=threads, **kw).run_reduce()
    base = tmp_path / "seqlen"
    s2m = MMapIndexedDataset(str(base / "seqlen_sample_to_metric"))
    np.testing.assert_array_equal(np.concatenate(s2m[0:len(s2m)]), ds.lens)
    i2s = MMapIndexedDataset(str(base / "seqlen_index_to_sample"))
    i2m = MMapIndexedDataset(str(base / "seqlen_index_to_metric"))
    vals = [int(i2m[r][0]) for r in range(len(i2m))]
    assert vals == sorted(set(ds.lens.tolist()))
    for r in range(len(i2s)):
        assert set(i2s[r].tolist()) == set(np.nonzero(ds.lens == vals[r])[0].tolist())
    merged = MMapIndexedDataset(str(base / "seqlen_index_to_sample_percentile_merged"))
    assert sum(len(x) for x in merged[0:len(merged)]) == len(ds)
    acc = MMapIndexedDataset(str(tmp_path / "vocab" / "vocab_metric_value"))[0]
    want = sum(torch.bincount(ds[i], minlength=8) for i in range(len(ds))).numpy()
    np.testing.assert_array_equal(acc, want)
    # the curriculum sampler reads the analyzer's index files directly
    cfg = {"seed": 3, "data_sampling": {"curriculum_learning": {"curriculum_metrics": {"seqlen": {
        "index_to_sample_path": str(base / "seqlen_index_to_sample"),
        "index_to_metric_path": str(base / "seqlen_index_to_metric"),
        "difficulty_type": "value", "clustering_type": "schedule_based", "min_difficulty": 10,
        "max_difficulty": 40, "schedule_type": "fixed_linear",
        "schedule_config": {"total_curriculum_step": 4, "difficulty_step": 1}}}}}}
    sampler = DeepSpeedDataSampler(cfg, len(ds), 4, 0, 1)
    first = next(iter(sampler))
    d = sampler.schedulers["seqlen"].get_current_difficulty()
    assert 10 <= d < 40 and all(ds.lens[i] <= d for i in first)
