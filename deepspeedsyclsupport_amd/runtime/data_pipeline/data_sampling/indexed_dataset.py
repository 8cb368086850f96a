"""Memory-mapped indexed datasets (reference `runtime/data_pipeline/data_sampling/indexed_dataset.py:369-620`,
Megatron's `.idx`/`.bin` "MMIDIDX" format, so files written by either side load in the other).

Layout of `<prefix>.idx` (little endian): magic b"MMIDIDX\\x00\\x00", u64 version (1), u8 dtype code, u64 number of
items, u64 number of document boundaries, then int32 sizes[n], int64 byte pointers[n], int64 doc_idx[docs].
`<prefix>.bin` holds the items back to back. Items are returned as zero-copy numpy views of the memory map.

Writing is vectorised: the builder accumulates sizes in a Python list and writes payload bytes straight to the
`.bin` file; `finalize` computes the pointers with one cumulative sum.
"""
import os
import shutil
import struct

import numpy as np
import torch

_HDR_MAGIC = b"MMIDIDX\x00\x00"

DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.float64, 7: np.double,
          8: np.uint16, 9: np.uint32, 10: np.uint64}


def code(dtype):
    dtype = np.dtype(dtype).type
    for k, v in DTYPES.items():
        if v == dtype:
            return k
    raise ValueError(dtype)


def index_file_path(prefix):
    return prefix + ".idx"


def data_file_path(prefix):
    return prefix + ".bin"


def best_fitting_dtype(vocab_size=None):
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def find_fit_int_dtype(min_value, max_value):
    """Smallest integer dtype holding [min_value, max_value] (reference `data_sampling/utils.py:13`)."""
    if min_value >= 0:
        for t in (np.uint8, np.uint16, np.uint32, np.uint64):
            if max_value <= np.iinfo(t).max:
                return t
    for t in (np.int8, np.int16, np.int32, np.int64):
        if np.iinfo(t).min <= min_value and max_value <= np.iinfo(t).max:
            return t
    return np.int64


class MMapIndexedDataset(torch.utils.data.Dataset):

    class Index:

        def __init__(self, path):
            with open(path, "rb") as f:
                assert f.read(9) == _HDR_MAGIC, f"{path}: not an MMIDIDX index file"
                (version, ) = struct.unpack("<Q", f.read(8))
                assert version == 1, f"{path}: unsupported index version {version}"
                (dcode, ) = struct.unpack("<B", f.read(1))
                self._dtype = DTYPES[dcode]
                self._len = struct.unpack("<Q", f.read(8))[0]
                self._doc_count = struct.unpack("<Q", f.read(8))[0]
                offset = f.tell()
            self._mmap = np.memmap(path, mode="r", order="C")
            buf = memoryview(self._mmap)
            self._sizes = np.frombuffer(buf, dtype=np.int32, count=self._len, offset=offset)
            self._pointers = np.frombuffer(buf, dtype=np.int64, count=self._len, offset=offset + self._sizes.nbytes)
            self._doc_idx = np.frombuffer(buf, dtype=np.int64, count=self._doc_count,
                                          offset=offset + self._sizes.nbytes + self._pointers.nbytes)

        @property
        def dtype(self):
            return self._dtype

        @property
        def sizes(self):
            return self._sizes

        @property
        def doc_idx(self):
            return self._doc_idx

        def __getitem__(self, i):
            return self._pointers[i], self._sizes[i]

        def __len__(self):
            return self._len

    def __init__(self, path, skip_warmup=True):
        super().__init__()
        self._do_init(path)

    def _do_init(self, path):
        self._path = path
        self._index = self.Index(index_file_path(path))
        nbytes = os.path.getsize(data_file_path(path))
        self._bin = np.memmap(data_file_path(path), mode="r", order="C") if nbytes else np.zeros(0, np.uint8)

    def __getstate__(self):
        return self._path

    def __setstate__(self, state):
        self._do_init(state)

    def __len__(self):
        return len(self._index)

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            ptr, size = self._index[idx]
            return np.frombuffer(self._bin, dtype=self._index.dtype, count=int(size), offset=int(ptr))
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            if step != 1:
                raise ValueError("slices into indexed datasets must be contiguous")
            ptr = int(self._index._pointers[start]) if stop > start else 0
            sizes = self._index._sizes[start:stop]
            flat = np.frombuffer(self._bin, dtype=self._index.dtype, count=int(sizes.sum()), offset=ptr)
            return np.split(flat, np.cumsum(sizes)[:-1])
        raise TypeError(f"unsupported index type {type(idx)}")

    def get(self, idx, offset=0, length=None):
        ptr, size = self._index[idx]
        if length is None:
            length = int(size) - offset
        item = np.dtype(self._index.dtype).itemsize
        return np.frombuffer(self._bin, dtype=self._index.dtype, count=length, offset=int(ptr) + offset * item)

    @property
    def sizes(self):
        return self._index.sizes

    def size(self, index):
        return int(self._index.sizes[index])

    @property
    def doc_idx(self):
        return self._index.doc_idx

    def get_doc_idx(self):
        return self._index._doc_idx

    def set_doc_idx(self, doc_idx):
        self._index._doc_idx = doc_idx

    @property
    def supports_prefetch(self):
        return False

    @property
    def dtype(self):
        return self._index.dtype

    @staticmethod
    def exists(path):
        return os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))


class MMapIndexedDatasetBuilder:

    def __init__(self, out_file, dtype=np.int64):
        self._file = open(out_file, "wb")
        self._dtype = np.dtype(dtype).type
        self._sizes = []
        self._doc_idx = [0]

    def add_item(self, tensor):
        arr = tensor.cpu().numpy() if torch.is_tensor(tensor) else np.asarray(tensor)
        self.add_item_numpy(arr)

    def add_item_numpy(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self._dtype).reshape(-1)
        self._file.write(arr.tobytes(order="C"))
        self._sizes.append(arr.size)

    def add_items_numpy(self, flat, sizes):
        """Append many items at once: `flat` is their concatenation, `sizes` the item lengths."""
        flat = np.ascontiguousarray(flat, dtype=self._dtype).reshape(-1)
        assert int(np.sum(sizes)) == flat.size
        self._file.write(flat.tobytes(order="C"))
        self._sizes.extend(int(s) for s in sizes)

    def end_document(self):
        self._doc_idx.append(len(self._sizes))

    def merge_file_(self, another_file):
        index = MMapIndexedDataset.Index(index_file_path(another_file))
        assert index.dtype == self._dtype, "merging datasets of different dtypes"
        base = len(self._sizes)
        self._sizes.extend(int(s) for s in index.sizes)
        self._doc_idx.extend(int(d) + base for d in index.doc_idx[1:])
        with open(data_file_path(another_file), "rb") as f:
            shutil.copyfileobj(f, self._file)

    def finalize(self, index_file):
        self._file.close()
        sizes = np.asarray(self._sizes, dtype=np.int64)
        pointers = np.zeros(len(sizes), dtype=np.int64)
        if len(sizes) > 1:
            np.cumsum(sizes[:-1] * np.dtype(self._dtype).itemsize, out=pointers[1:])
        with open(index_file, "wb") as f:
            f.write(_HDR_MAGIC)
            f.write(struct.pack("<Q", 1))
            f.write(struct.pack("<B", code(self._dtype)))
            f.write(struct.pack("<Q", len(sizes)))
            f.write(struct.pack("<Q", len(self._doc_idx)))
            f.write(sizes.astype(np.int32).tobytes(order="C"))
            f.write(pointers.tobytes(order="C"))
            f.write(np.asarray(self._doc_idx, dtype=np.int64).tobytes(order="C"))


def make_builder(out_file, impl="mmap", vocab_size=None, dtype=None):
    assert impl == "mmap", "only the mmap implementation is provided"
    return MMapIndexedDatasetBuilder(out_file, dtype=dtype or best_fitting_dtype(vocab_size))


def make_dataset(path, impl="mmap", skip_warmup=True):
    if not MMapIndexedDataset.exists(path):
        raise FileNotFoundError(f"dataset {path}.idx/.bin not found")
    return MMapIndexedDataset(path, skip_warmup)


def create_mmap_dataset_builder(fname, dtype):
    return MMapIndexedDatasetBuilder(data_file_path(fname), dtype=dtype)


def close_mmap_dataset_builder(builder, fname):
    builder.end_document()
    builder.finalize(index_file_path(fname))
