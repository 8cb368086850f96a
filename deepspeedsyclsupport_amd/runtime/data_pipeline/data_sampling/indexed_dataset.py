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


# ------------------------------------------------------------------------------------------------ legacy formats
# "lazy" / "cached": the older Megatron / fairseq index ("TNTIDX" header, big-endian-free struct fields, then the
# dimension offsets, data offsets, sizes and document index as int64 arrays); the data file is the items back to back.
_LEGACY_MAGIC = b"TNTIDX\x00\x00"


def read_longs(f, n):
    a = np.empty(n, dtype=np.int64)
    f.readinto(a)
    return a


def write_longs(f, a):
    f.write(np.array(a, dtype=np.int64))


def create_doc_idx(sizes):
    """Document boundaries from item sizes: an item of size 0 ends a document."""
    doc_idx = [0]
    for i, s in enumerate(sizes):
        if s == 0:
            doc_idx.append(i + 1)
    return doc_idx


def exscan_from_cumsum_(arr):
    """In place: inclusive prefix sum -> exclusive prefix sum (shift right, first element 0)."""
    if arr.size > 1:
        arr[1:] = arr[:-1]
    if arr.size > 0:
        arr[0] = 0


def get_pointers_with_total(sizes, elemsize, dtype):
    """(byte offset of every item, total bytes) from item sizes in elements."""
    pointers = np.array(sizes, dtype=dtype)
    np.cumsum(pointers, axis=0, out=pointers)
    total = int(pointers[-1]) * elemsize if len(sizes) else 0
    exscan_from_cumsum_(pointers)
    pointers *= elemsize
    return pointers, total


class IndexedDataset(torch.utils.data.Dataset):
    """Reader of the legacy index format; items are read from the data file on access ("lazy")."""

    def __init__(self, path):
        super().__init__()
        self.path = path
        self.data_file = None
        self.read_index(path)

    def read_index(self, path):
        import struct
        with open(index_file_path(path), "rb") as f:
            magic = f.read(8)
            assert magic == _LEGACY_MAGIC, "Index file doesn't match expected format. Make sure that --dataset-impl " \
                "is configured properly."
            assert struct.unpack("<Q", f.read(8)) == (1, )
            dcode, self.element_size = struct.unpack("<QQ", f.read(16))
            self.dtype = DTYPES[dcode]
            self._len, self.s = struct.unpack("<QQ", f.read(16))
            self.doc_count = struct.unpack("<Q", f.read(8))[0]
            self.dim_offsets = read_longs(f, self._len + 1)
            self.data_offsets = read_longs(f, self._len + 1)
            self.sizes = read_longs(f, self.s)
            self.doc_idx = read_longs(f, self.doc_count)

    def read_data(self, path):
        self.data_file = open(data_file_path(path), "rb", buffering=0)

    def check_index(self, i):
        if i < 0 or i >= self._len:
            raise IndexError("index out of range")

    def __del__(self):
        if self.data_file:
            self.data_file.close()

    def __getitem__(self, idx):
        if not self.data_file:
            self.read_data(self.path)
        if isinstance(idx, int):
            self.check_index(idx)
            shape = self.sizes[self.dim_offsets[idx]:self.dim_offsets[idx + 1]]
            a = np.empty(shape, dtype=self.dtype)
            self.data_file.seek(int(self.data_offsets[idx]) * self.element_size)
            self.data_file.readinto(a)
            return a
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            if step != 1:
                raise ValueError("Slices into indexed_dataset must be contiguous")
            sizes = self.sizes[self.dim_offsets[start]:self.dim_offsets[stop]]
            a = np.empty(int(sum(sizes)), dtype=self.dtype)
            self.data_file.seek(int(self.data_offsets[start]) * self.element_size)
            self.data_file.readinto(a)
            return np.split(a, np.cumsum(sizes)[:-1])
        raise TypeError(f"unsupported index {idx!r}")

    def __len__(self):
        return self._len

    def num_tokens(self, index):
        return self.sizes[index]

    def size(self, index):
        return self.sizes[index]

    @staticmethod
    def exists(path):
        return os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))

    @property
    def supports_prefetch(self):
        return False


class IndexedCachedDataset(IndexedDataset):
    """Legacy format with `prefetch(indices)`: the requested items are read once into one array and served from
    it."""

    def __init__(self, path):
        super().__init__(path)
        self.cache = None
        self.cache_index = {}

    @property
    def supports_prefetch(self):
        return True

    def prefetch(self, indices):
        if all(i in self.cache_index for i in indices):
            return
        if not self.data_file:
            self.read_data(self.path)
        indices = sorted(set(indices))
        total = sum(int(self.data_offsets[i + 1] - self.data_offsets[i]) for i in indices)
        self.cache = np.empty(total, dtype=self.dtype)
        self.cache_index.clear()
        ptx = 0
        for i in indices:
            self.cache_index[i] = ptx
            size = int(self.data_offsets[i + 1] - self.data_offsets[i])
            self.data_file.seek(int(self.data_offsets[i]) * self.element_size)
            self.data_file.readinto(self.cache[ptx:ptx + size])
            ptx += size
        if self.data_file:
            self.data_file.close()
            self.data_file = None

    def __getitem__(self, idx):
        if isinstance(idx, int) and idx in self.cache_index:
            self.check_index(idx)
            shape = self.sizes[self.dim_offsets[idx]:self.dim_offsets[idx + 1]]
            ptx = self.cache_index[idx]
            return self.cache[ptx:ptx + int(np.prod(shape))].reshape(shape).copy()
        if isinstance(idx, slice):
            return [self[i] for i in range(*idx.indices(len(self)))]
        return super().__getitem__(idx)


class IndexedDatasetBuilder:
    """Writer of the legacy format."""
    element_sizes = {np.uint8: 1, np.int8: 1, np.int16: 2, np.int32: 4, np.int64: 8, np.float64: 8, np.double: 8}

    def __init__(self, out_file, dtype=np.int32):
        self.out_file = open(out_file, "wb")
        self.dtype = dtype
        self.data_offsets, self.dim_offsets, self.sizes, self.doc_idx = [0], [0], [], [0]
        self.element_size = np.dtype(dtype).itemsize

    def add_item(self, tensor):
        arr = np.asarray(tensor.numpy() if torch.is_tensor(tensor) else tensor, dtype=self.dtype)
        n = self.out_file.write(arr.tobytes())
        self.data_offsets.append(self.data_offsets[-1] + n // self.element_size)
        self.sizes.extend(arr.shape)
        self.dim_offsets.append(self.dim_offsets[-1] + arr.ndim)

    def end_document(self):
        self.doc_idx.append(len(self.sizes))

    def merge_file_(self, another_file):
        other = IndexedDataset(another_file)
        assert other.dtype == self.dtype
        doc_offset = len(self.sizes)
        begin = self.data_offsets[-1]
        self.data_offsets.extend(begin + int(o) for o in other.data_offsets[1:])
        self.sizes.extend(int(x) for x in other.sizes)
        begin = self.dim_offsets[-1]
        self.dim_offsets.extend(begin + int(o) for o in other.dim_offsets[1:])
        self.doc_idx.extend(doc_offset + int(d) for d in other.doc_idx[1:])
        with open(data_file_path(another_file), "rb") as f:
            while True:
                data = f.read(1 << 20)
                if not data:
                    break
                self.out_file.write(data)

    def finalize(self, index_file):
        import struct
        self.out_file.close()
        with open(index_file, "wb") as index:
            index.write(_LEGACY_MAGIC)
            index.write(struct.pack("<Q", 1))
            index.write(struct.pack("<QQ", code(self.dtype), self.element_size))
            index.write(struct.pack("<QQ", len(self.data_offsets) - 1, len(self.sizes)))
            index.write(struct.pack("<Q", len(self.doc_idx)))
            write_longs(index, self.dim_offsets)
            write_longs(index, self.data_offsets)
            write_longs(index, self.sizes)
            write_longs(index, self.doc_idx)


# ------------------------------------------------------------------------------------------------ factories
def get_available_dataset_impl():
    return ["lazy", "cached", "mmap"]


def infer_dataset_impl(path):
    """"cached" for a legacy index, "mmap" for the memory-mapped one, None when the index is neither / absent."""
    if not IndexedDataset.exists(path):
        print(f"Dataset does not exist: {path}")
        print("Path should be a basename that both .idx and .bin can be appended to get full filenames.")
        return None
    with open(index_file_path(path), "rb") as f:
        magic = f.read(8)
    if magic == _LEGACY_MAGIC:
        return "cached"
    if magic == _HDR_MAGIC[:8]:
        return "mmap"
    return None


def dataset_exists(path, impl):
    return MMapIndexedDataset.exists(path) if impl == "mmap" else IndexedDataset.exists(path)


def make_builder(out_file, impl="mmap", vocab_size=None, dtype=None):
    if impl == "mmap":
        return MMapIndexedDatasetBuilder(out_file, dtype=dtype or best_fitting_dtype(vocab_size))
    return IndexedDatasetBuilder(out_file) if dtype is None else IndexedDatasetBuilder(out_file, dtype=dtype)


def make_dataset(path, impl="mmap", skip_warmup=True):
    if not IndexedDataset.exists(path):
        raise FileNotFoundError(f"dataset {path}.idx/.bin not found")
    if impl == "infer":
        impl = infer_dataset_impl(path)
    if impl == "lazy":
        return IndexedDataset(path)
    if impl == "cached":
        return IndexedCachedDataset(path)
    if impl == "mmap":
        return MMapIndexedDataset(path, skip_warmup)
    raise ValueError(f"Unknown dataset implementation: {impl}")


def create_mmap_dataset_builder(fname, dtype):
    return MMapIndexedDatasetBuilder(data_file_path(fname), dtype=dtype)


def close_mmap_dataset_builder(builder, fname):
    builder.end_document()
    builder.finalize(index_file_path(fname))
