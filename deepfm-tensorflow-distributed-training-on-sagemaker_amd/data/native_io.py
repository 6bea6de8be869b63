"""ctypes binding of ``_lib/libhipfm_io.so`` (csrc/io/hfm_io.cpp): the native TFRecord /
Example / libsvm reader, threaded deterministic batch loader, CRC32C and writers."""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Iterator, Optional, Sequence, Tuple

import numpy as np

from ..ops.build import IO_SO, build_io

_lib = None
_lock = threading.Lock()

FMT_TFRECORD, FMT_LIBSVM = 0, 1


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(IO_SO):
                build_io()
            L = C.CDLL(IO_SO)
            vp, ci, cl = C.c_void_p, C.c_int, C.c_long
            L.hfmio_last_error.restype = C.c_char_p
            L.hfmio_crc32c.argtypes = [vp, C.c_size_t]
            L.hfmio_crc32c.restype = C.c_uint32
            L.hfmio_crc32c_extend.argtypes = [C.c_uint32, vp, C.c_size_t]
            L.hfmio_crc32c_extend.restype = C.c_uint32
            L.hfmio_masked_crc32c.argtypes = [vp, C.c_size_t]
            L.hfmio_masked_crc32c.restype = C.c_uint32
            L.hfmio_decode_example.argtypes = [vp, C.c_size_t, ci, vp, vp, vp]
            L.hfmio_decode_example.restype = ci
            L.hfmio_loader_create.argtypes = [C.POINTER(C.c_char_p), ci, ci, ci, ci, ci, ci, ci, ci,
                                              ci, ci, C.c_int64, ci]
            L.hfmio_loader_create.restype = vp
            L.hfmio_loader_next.argtypes = [vp, vp, vp, vp]
            L.hfmio_loader_next.restype = ci
            L.hfmio_loader_next32.argtypes = [vp, vp, vp, vp]
            L.hfmio_loader_next32.restype = ci
            L.hfmio_loader_next32c.argtypes = [vp, vp, vp, vp, vp]
            L.hfmio_loader_next32c.restype = ci
            L.hfmio_loader_start_ring.argtypes = [vp, ci, vp, vp, vp, ci]
            L.hfmio_loader_start_ring.restype = ci
            L.hfmio_loader_ring_take.argtypes = [vp, vp, vp]
            L.hfmio_loader_ring_take.restype = ci
            L.hfmio_loader_ring_give.argtypes = [vp, ci]
            L.hfmio_loader_ring_give.restype = None
            L.hfmio_loader_destroy.argtypes = [vp]
            L.hfmio_loader_create_raw.argtypes = [C.POINTER(C.c_char_p), ci, ci, ci, ci, ci, ci, ci, ci, ci]
            L.hfmio_loader_create_raw.restype = vp
            L.hfmio_loader_next_raw.argtypes = [vp, vp, C.c_size_t, vp, vp]
            L.hfmio_loader_next_raw.restype = ci
            L.hfmio_loader_start_ring_raw.argtypes = [vp, ci, vp, C.c_size_t, vp]
            L.hfmio_loader_start_ring_raw.restype = ci
            L.hfmio_loader_set_copy_threads.argtypes = [vp, ci]
            L.hfmio_loader_set_copy_threads.restype = None
            L.hfmio_write_examples.argtypes = [C.c_char_p, vp, vp, vp, cl, ci, ci]
            L.hfmio_write_examples.restype = ci
            L.hfmio_libsvm_to_tfrecord.argtypes = [C.c_char_p, C.c_char_p, ci]
            L.hfmio_libsvm_to_tfrecord.restype = cl
            L.hfmio_count_records.argtypes = [C.c_char_p, ci, ci]
            L.hfmio_count_records.restype = cl
            _lib = L
    return _lib


def _err() -> str:
    return lib().hfmio_last_error().decode(errors="replace")


def crc32c(data: bytes) -> int:
    return lib().hfmio_crc32c(data, len(data))


def crc32c_extend(crc: int, data: bytes) -> int:
    """crc32c(a + b) == crc32c_extend(crc32c(a), b)"""
    return lib().hfmio_crc32c_extend(crc, data, len(data))


def mask_crc(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    return lib().hfmio_masked_crc32c(data, len(data))


def decode_example(data: bytes, F: int):
    lab = np.zeros(1, np.float32)
    ids = np.zeros(F, np.int64)
    vals = np.zeros(F, np.float32)
    rc = lib().hfmio_decode_example(data, len(data), F, lab.ctypes.data, ids.ctypes.data,
                                    vals.ctypes.data)
    if rc != 0:
        raise ValueError("Example does not match the fixed schema")
    return float(lab[0]), ids, vals


def write_examples(path: str, labels: np.ndarray, ids: np.ndarray, vals: np.ndarray,
                   append: bool = False) -> None:
    labels = np.ascontiguousarray(labels, np.float32)
    ids = np.ascontiguousarray(ids, np.int64)
    vals = np.ascontiguousarray(vals, np.float32)
    n, F = ids.shape
    if lib().hfmio_write_examples(path.encode(), labels.ctypes.data, ids.ctypes.data,
                                  vals.ctypes.data, n, F, 1 if append else 0) != 0:
        raise IOError(_err())


def libsvm_to_tfrecord(src: str, dst: str, field_size: int) -> int:
    n = lib().hfmio_libsvm_to_tfrecord(src.encode(), dst.encode(), field_size)
    if n < 0:
        raise IOError(_err())
    return n


def count_records(path: str, fmt: int = FMT_TFRECORD, verify: bool = True) -> int:
    n = lib().hfmio_count_records(path.encode(), fmt, 1 if verify else 0)
    if n < 0:
        raise IOError(_err())
    return n


def _addr(a) -> int:
    return a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr()


def _dtype_of(a) -> int:
    return a.dtype.itemsize if isinstance(a, np.ndarray) else a.element_size()


def mask_fields(mask: int, F: int):
    """The shipped (non-constant) fields of a compact-values mask, in column order."""
    return [f for f in range(F) if (mask >> f) & 1]


def expand_values(vals_c, rows: int, F: int, mask: int) -> np.ndarray:
    """Host inverse of the compact value format: [rows, F] float32 with the shipped columns in
    place and 1.0 elsewhere (the device does the same in ops.kernels.expand_vals)."""
    cols = mask_fields(mask, F)
    out = np.ones((rows, F), np.float32)
    src = np.asarray(vals_c).reshape(-1)[:rows * len(cols)]
    out[:, cols] = src.reshape(rows, len(cols))
    return out


class NativeLoader:
    """Iterator of (labels f32[B], ids i64[B,F], vals f32[B,F]) numpy batches.

    ``record_shard=(n, i)`` reproduces ``dataset.shard(n, i)`` on the concatenated record
    stream (reference semantics); without it the files are read in parallel by ``threads``
    workers with a deterministic round-robin interleave of 1024-record chunks.
    ``id_limit`` (> 0, the table size V): a record with an id outside [0, V) fails the read with
    an error naming the file and the record index (the device gathers rows unchecked)."""

    def __init__(self, paths: Sequence[str], field_size: int, batch_size: int,
                 fmt: int = FMT_TFRECORD, drop_remainder: bool = True, threads: int = 4,
                 record_shard: Tuple[int, int] = (1, 0), verify_crc: bool = True,
                 queue_depth: int = 4, id_limit: int = 0, copy_threads: Optional[int] = None,
                 ids32: bool = False, raw: bool = False, device_crc: bool = False):
        self.paths = [str(p) for p in paths]
        self.F, self.B = int(field_size), int(batch_size)
        # raw (TFRecord only): the workers frame records and check CRCs, batches carry the
        # serialized Examples for the GPU decoder (ops.kernels.decode_examples)
        self.raw = bool(raw)
        # device_crc (raw, verify_crc): the workers check only each record's length CRC and ship
        # the record with its 4-byte data CRC, which the decode kernel verifies (decode_examples
        # crc=True) -- no per-byte work on the host
        self.device_crc = self.raw and bool(device_crc) and bool(verify_crc)
        arr = (C.c_char_p * max(1, len(self.paths)))(*[p.encode() for p in self.paths])
        if self.raw:
            if fmt != FMT_TFRECORD:
                raise ValueError("raw records are TFRecord Examples")
            vmode = 2 if self.device_crc else (1 if verify_crc else 0)
            self._h = lib().hfmio_loader_create_raw(arr, len(self.paths), self.F, self.B,
                                                    1 if drop_remainder else 0, threads, record_shard[0],
                                                    record_shard[1], vmode, queue_depth)
        else:
            self._h = lib().hfmio_loader_create(arr, len(self.paths), fmt, self.F, self.B,
                                                1 if drop_remainder else 0, threads, record_shard[0],
                                                record_shard[1], 1 if verify_crc else 0, queue_depth,
                                                int(id_limit), 1 if ids32 else 0)
        # batches are assembled from the workers' chunks by a copy pool (the consumer alone
        # capped ingest near 49 M rows/s at B = 16384; on a 16-core share of an EPYC 9575F: 16
        # decode threads + 1 / 4 / 8 copy threads = 45 / 70 / 97 M rows/s with int64 chunks
        # narrowed while copying -- ``ids32`` narrows at decode time instead)
        ct = copy_threads if copy_threads is not None else max(1, min(8, int(threads) // 2))
        lib().hfmio_loader_set_copy_threads(self._h, int(ct))
        self._done = False

    def next_into(self, labels, ids, vals) -> int:
        """Fill caller buffers (numpy arrays or pinned CPU torch tensors); ``ids`` int64, or int32
        (narrowed in the loader thread, checked to fit); returns rows (0 at end)."""
        if self._done:
            return 0
        fn = lib().hfmio_loader_next32 if _dtype_of(ids) == 4 else lib().hfmio_loader_next
        r = fn(self._h, _addr(labels), _addr(ids), _addr(vals))
        if r < 0:
            raise IOError(_err())
        if r == 0:
            self._done = True
        return r

    def next_into_compact(self, labels, ids32, vals_c) -> Tuple[int, int]:
        """``next_into`` with int32 ids and compact values: ``vals_c`` (>= B*F floats) receives
        only the columns of the fields whose values are not all exactly 1.0 in the batch, [rows,
        nc] row-major in field order; returns (rows, mask) with bit f of ``mask`` set for each
        shipped field f (nc = popcount(mask)).  Lossless: the other fields' values are 1.0f in
        every row (``expand_values``).  Needs F <= 64."""
        if self._done:
            return 0, 0
        assert _dtype_of(ids32) == 4 and self.F <= 64
        m = C.c_uint64(0)
        r = lib().hfmio_loader_next32c(self._h, _addr(labels), _addr(ids32), _addr(vals_c), C.addressof(m))
        if r < 0:
            raise IOError(_err())
        if r == 0:
            self._done = True
        return r, int(m.value)

    def start_ring(self, bufs, compact: bool = False) -> None:
        """Assemble ahead into ``bufs`` = [(labels, ids32, vals), ...] (>= 2 slots; pinned CPU
        tensors or numpy arrays that outlive the loader's use of them) on a C++ assembler thread,
        in cyclic slot order; ``compact``: ``vals`` get the compact columns (next_into_compact).
        Then ``ring_take`` / ``ring_give`` instead of ``next_into``."""
        n = len(bufs)
        arr = lambda xs: (C.c_void_p * n)(*[_addr(x) for x in xs])  # noqa: E731
        for lab, ids, vals in bufs:
            assert _dtype_of(ids) == 4, "the assembly ring writes int32 ids"
        self._ring_keep = bufs
        if lib().hfmio_loader_start_ring(self._h, n, arr([b[0] for b in bufs]), arr([b[1] for b in bufs]),
                                         arr([b[2] for b in bufs]), 1 if compact else 0) != 0:
            raise IOError(_err())

    def next_raw_into(self, raw, offs) -> Tuple[int, int]:
        """Raw loader: the next batch's record bytes into ``raw`` (uint8, its size is the capacity)
        and B + 1 int32 start offsets into ``offs``; returns (rows, bytes), rows 0 at end."""
        if self._done:
            return 0, 0
        nb = C.c_uint64(0)
        cap = raw.numel() if hasattr(raw, "numel") else raw.size
        r = lib().hfmio_loader_next_raw(self._h, _addr(raw), cap, _addr(offs), C.addressof(nb))
        if r < 0:
            raise IOError(_err())
        if r == 0:
            self._done = True
        return r, int(nb.value)

    def start_ring_raw(self, bufs) -> None:
        """Raw loader: assemble ahead into ``bufs`` = [(raw uint8 [cap], offs int32 [B + 1]), ...]
        (equal capacities) on the C++ assembler thread; ``ring_take`` then returns (rows, slot,
        bytes)."""
        n = len(bufs)
        cap = min(int(r.numel()) for r, _ in bufs)
        self._ring_keep = bufs
        if lib().hfmio_loader_start_ring_raw(self._h, n, (C.c_void_p * n)(*[_addr(r) for r, _ in bufs]), cap,
                                             (C.c_void_p * n)(*[_addr(o) for _, o in bufs])) != 0:
            raise IOError(_err())

    def ring_take(self) -> Tuple[int, int, int]:
        """(rows, slot, mask) of the next assembled slot (blocks; the GIL is released); rows 0 at
        the end.  The slot's buffers are the caller's until ``ring_give(slot)``."""
        slot, m = C.c_int(0), C.c_uint64(0)
        r = lib().hfmio_loader_ring_take(self._h, C.addressof(slot), C.addressof(m))
        if r < 0:
            raise IOError(_err())
        return r, slot.value, int(m.value)

    def ring_give(self, slot: int) -> None:
        lib().hfmio_loader_ring_give(self._h, int(slot))

    def __iter__(self) -> Iterator[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
        while True:
            lab = np.empty(self.B, np.float32)
            ids = np.empty((self.B, self.F), np.int64)
            vals = np.empty((self.B, self.F), np.float32)
            r = self.next_into(lab, ids, vals)
            if r == 0:
                return
            yield lab[:r], ids[:r], vals[:r]

    def close(self):
        if self._h:
            lib().hfmio_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
