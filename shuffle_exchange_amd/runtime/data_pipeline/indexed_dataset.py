"""Memory-mapped token datasets in the Megatron ``.bin`` / ``.idx`` format.

Parity: reference runtime/data_pipeline/data_sampling/indexed_dataset.py -- ``MMapIndexedDataset``
:369 (with ``Index`` reader/writer :371-470), ``MMapIndexedDatasetBuilder`` :575, ``make_builder`` /
``make_dataset`` / ``data_file_path`` / ``index_file_path``, dtype codes :102-111. The on-disk format
is byte-compatible so existing corpora load unchanged:

  idx: b"MMIDIDX\\x00\\x00" | <Q version=1 | <B dtype code | <Q n_items | <Q n_docs |
       int32 sizes[n_items] | int64 byte pointers[n_items] | int64 doc_idx[n_docs]
  bin: the items' tokens back to back.

Reading is zero-copy (``np.memmap`` + ``np.frombuffer`` views); ``get(i, offset, length)`` slices a
sample without touching the rest, which is what the data analyzer and sequence-packing samplers
need for multi-TB corpora on the host of an MI355X node.
"""
import os
import shutil
import struct

import numpy as np
import torch

_MAGIC = b"MMIDIDX\x00\x00"
DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.uint16, 7: np.uint32,
          8: np.uint64}
_TORCH = {np.uint8: torch.uint8, np.int8: torch.int8, np.int16: torch.int16, np.int32: torch.int32,
          np.int64: torch.int64}


def code(dtype):
    dt = np.dtype(dtype).type if not isinstance(dtype, torch.dtype) else \
        {v: k for k, v in _TORCH.items()}[dtype]
    for k, v in DTYPES.items():
        if v == dt:
            return k
    raise ValueError(f"unsupported dtype {dtype}")


def best_fitting_dtype(vocab_size=None):
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def index_file_path(prefix):
    return prefix + ".idx"


def data_file_path(prefix):
    return prefix + ".bin"


def exists(prefix):
    return os.path.exists(index_file_path(prefix)) and os.path.exists(data_file_path(prefix))


class MMapIndexedDataset(torch.utils.data.Dataset):
    class Index:
        _HDR_MAGIC = _MAGIC

        def __init__(self, path, skip_warmup=True):
            with open(path, "rb") as f:
                assert f.read(9) == _MAGIC, f"{path}: not an MMIDIDX index file"
                (version,) = struct.unpack("<Q", f.read(8))
                assert version == 1, f"{path}: index version {version}"
                (dt,) = struct.unpack("<B", f.read(1))
                self._dtype = DTYPES[dt]
                self._len, self._doc_count = struct.unpack("<QQ", f.read(16))
                offset = f.tell()
            self._buf = np.memmap(path, mode="r", order="C")
            self._sizes = np.frombuffer(self._buf, dtype=np.int32, count=self._len, offset=offset)
            self._pointers = np.frombuffer(self._buf, dtype=np.int64, count=self._len,
                                           offset=offset + self._sizes.nbytes)
            self._doc_idx = np.frombuffer(self._buf, dtype=np.int64, count=self._doc_count,
                                          offset=offset + self._sizes.nbytes + self._pointers.nbytes)

        @staticmethod
        def write(path, dtype, sizes, doc_idx):
            sizes = np.asarray(sizes, dtype=np.int32)
            item = np.dtype(dtype).itemsize
            pointers = np.zeros(len(sizes), dtype=np.int64)
            if len(sizes) > 1:
                np.cumsum(sizes[:-1].astype(np.int64) * item, out=pointers[1:])
            with open(path, "wb") as f:
                f.write(_MAGIC)
                f.write(struct.pack("<Q", 1))
                f.write(struct.pack("<B", code(dtype)))
                f.write(struct.pack("<QQ", len(sizes), len(doc_idx)))
                f.write(sizes.tobytes(order="C"))
                f.write(pointers.tobytes(order="C"))
                f.write(np.asarray(doc_idx, dtype=np.int64).tobytes(order="C"))

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
        self._path = path
        self._index = self.Index(index_file_path(path))
        self._bin = np.memmap(data_file_path(path), mode="r", order="C")

    def __getstate__(self):
        return self._path

    def __setstate__(self, path):
        self.__init__(path)

    def __len__(self):
        return len(self._index)

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            ptr, size = self._index[idx]
            return np.frombuffer(self._bin, dtype=self._index.dtype, count=int(size), offset=int(ptr))
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            assert step == 1, "slices must be contiguous"
            ptr = self._index._pointers[start]
            sizes = self._index._sizes[start:stop]
            flat = np.frombuffer(self._bin, dtype=self._index.dtype, count=int(sizes.sum()), offset=int(ptr))
            return np.split(flat, np.cumsum(sizes)[:-1])
        raise TypeError(f"index type {type(idx)}")

    def get(self, idx, offset=0, length=None):
        ptr, size = self._index[idx]
        length = int(size) - offset if length is None else length
        ptr = int(ptr) + offset * np.dtype(self._index.dtype).itemsize
        return np.frombuffer(self._bin, dtype=self._index.dtype, count=length, offset=ptr)

    @property
    def sizes(self):
        return self._index.sizes

    @property
    def doc_idx(self):
        return self._index.doc_idx

    @property
    def dtype(self):
        return self._index.dtype

    @staticmethod
    def exists(path):
        return exists(path)


class MMapIndexedDatasetBuilder:
    def __init__(self, out_file, dtype=np.int64):
        self._data = open(out_file, "wb")
        self._dtype = np.dtype(dtype).type if not isinstance(dtype, torch.dtype) else \
            {v: k for k, v in _TORCH.items()}[dtype]
        self._sizes, self._doc_idx = [], [0]

    def add_item(self, tensor):
        a = np.asarray(tensor.numpy() if torch.is_tensor(tensor) else tensor, dtype=self._dtype)
        self._data.write(a.tobytes(order="C"))
        self._sizes.append(a.size)

    def add_item_numpy(self, a):
        self.add_item(a)

    def add_items(self, arrays):
        for a in arrays:
            self.add_item(a)

    def end_document(self):
        self._doc_idx.append(len(self._sizes))

    def merge_file_(self, another_prefix):
        idx = MMapIndexedDataset.Index(index_file_path(another_prefix))
        assert idx.dtype == self._dtype, "dtype mismatch"
        off = len(self._sizes)
        self._sizes.extend(idx.sizes.tolist())
        self._doc_idx.extend((off + idx.doc_idx[1:]).tolist())
        with open(data_file_path(another_prefix), "rb") as f:
            shutil.copyfileobj(f, self._data)

    def finalize(self, index_file):
        self._data.close()
        MMapIndexedDataset.Index.write(index_file, self._dtype, self._sizes, self._doc_idx)


def make_builder(out_file, impl="mmap", vocab_size=None, dtype=None):
    assert impl == "mmap", "only the mmap implementation is provided"
    return MMapIndexedDatasetBuilder(out_file, dtype=dtype or best_fitting_dtype(vocab_size))


def make_dataset(path, impl="mmap", skip_warmup=True):
    assert impl in ("mmap", "infer"), "only the mmap implementation is provided"
    return MMapIndexedDataset(path, skip_warmup)
