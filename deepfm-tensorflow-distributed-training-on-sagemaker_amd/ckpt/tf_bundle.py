"""TensorFlow ``tensor_bundle`` checkpoint writer/reader without TensorFlow.

A TF1 checkpoint ``model.ckpt-<step>`` is
  * ``model.ckpt-<step>.data-0000r-of-0000N`` — raw little-endian tensor bytes, back to back;
    every variable lives whole in one of the N data shards (TF1 PS jobs write one shard per
    parameter-server task; ``ShardWriter`` lets each rank write its own);
  * ``model.ckpt-<step>.index`` — a LevelDB-format SSTable mapping tensor name ->
    ``BundleEntryProto{dtype, shape, shard_id, offset, size, crc32c}``, plus the header entry
    under the empty key -> ``BundleHeaderProto{num_shards, endianness, version}``;
  * ``checkpoint`` — text proto naming the latest prefix (Estimator's CheckpointState).
Keys are written in bytewise order; blocks use LevelDB prefix compression with restart points
every 16 entries, no compression, and a masked-CRC32C trailer.

This lets a hipfm model be exported with the reference's variable names / TF layouts
(``fm_bias``, ``fm_w``, ``fm_v``, ``Deep-part/mlp{i}/weights`` [in,out], optimizer slots
``<var>/Adam``...) and reads such checkpoints back.  Verified structurally (round trip, CRCs,
SSTable invariants); no TensorFlow is available here to load it (parity unpinned).
"""
from __future__ import annotations

import os
import struct
from typing import BinaryIO, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from ..data.tfrecord import _fields, _varint, masked_crc32c

try:
    from ..data import native_io as _nio
except Exception:  # pragma: no cover
    _nio = None

DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_BFLOAT16 = 1, 2, 3, 9, 14
_NP2DT = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): DT_DOUBLE,
          np.dtype(np.int32): DT_INT32, np.dtype(np.int64): DT_INT64}
_DT2NP = {v: k for k, v in _NP2DT.items()}
TABLE_MAGIC = 0xDB4775248B80FB57
BLOCK_SIZE = 262144
RESTART_INTERVAL = 16


def _mcrc(b: bytes) -> int:
    if _nio is not None:
        try:
            return _nio.masked_crc32c(b)
        except Exception:
            pass
    return masked_crc32c(b)


def _crc_raw(b: bytes) -> int:
    """unmasked crc32c (the BundleEntryProto.crc32c field stores the MASKED value)."""
    return _mcrc(b)


# ------------------------------------------------------------------------------ protos
def _ld(f: int, payload: bytes) -> bytes:
    return _varint((f << 3) | 2) + _varint(len(payload)) + payload


def _vi(f: int, v: int) -> bytes:
    return _varint(f << 3) + _varint(v)


def _fx32(f: int, v: int) -> bytes:
    return _varint((f << 3) | 5) + struct.pack("<I", v & 0xFFFFFFFF)


def bundle_entry(dtype: int, shape: Tuple[int, ...], offset: int, size: int, crc: int,
                 shard_id: int = 0) -> bytes:
    shp = b"".join(_ld(2, _vi(1, d)) for d in shape)   # TensorShapeProto.dim{size}
    out = _vi(1, dtype) + _ld(2, shp)
    if shard_id:
        out += _vi(3, shard_id)
    if offset:
        out += _vi(4, offset)
    out += _vi(5, size) + _fx32(6, crc)
    return out


def bundle_header(num_shards: int = 1) -> bytes:
    return _vi(1, num_shards) + _ld(3, _vi(1, 1))       # endianness LITTLE(0) omitted; producer 1


def parse_entry(b: bytes) -> dict:
    d = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": 0}
    for f, wt, v in _fields(b):
        if f == 1:
            d["dtype"] = v
        elif f == 2:
            for f2, _, dim in _fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, x in _fields(dim):
                        if f3 == 1:
                            size = x
                    d["shape"].append(size)
        elif f == 3:
            d["shard_id"] = v
        elif f == 4:
            d["offset"] = v
        elif f == 5:
            d["size"] = v
        elif f == 6:
            d["crc32c"] = struct.unpack("<I", v)[0]
    return d


# ------------------------------------------------------------------------------ SSTable
class _BlockBuilder:
    def __init__(self):
        self.buf = bytearray()
        self.restarts = [0]
        self.count = 0
        self.last = b""

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.count < RESTART_INTERVAL:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.count = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.count += 1

    def finish(self) -> bytes:
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def empty(self) -> bool:
        return not self.buf


def _handle(off: int, size: int) -> bytes:
    return _varint(off) + _varint(size)


def write_sstable(path: str, items: List[Tuple[bytes, bytes]]) -> None:
    items = sorted(items, key=lambda kv: kv[0])
    with open(path, "wb") as f:
        off = 0
        index = _BlockBuilder()

        def flush(block: _BlockBuilder, last_key: bytes):
            nonlocal off
            data = block.finish()
            trailer = b"\x00" + struct.pack("<I", _mcrc(data + b"\x00"))
            f.write(data + trailer)
            index.add(last_key, _handle(off, len(data)))
            off += len(data) + 5

        blk = _BlockBuilder()
        last = b""
        for k, v in items:
            blk.add(k, v)
            last = k
            if blk.size() >= BLOCK_SIZE:
                flush(blk, last)
                blk = _BlockBuilder()
        if not blk.empty():
            flush(blk, last)
        # empty metaindex block
        meta = _BlockBuilder().finish()
        meta_h = _handle(off, len(meta))
        f.write(meta + b"\x00" + struct.pack("<I", _mcrc(meta + b"\x00")))
        off += len(meta) + 5
        idx = index.finish()
        idx_h = _handle(off, len(idx))
        f.write(idx + b"\x00" + struct.pack("<I", _mcrc(idx + b"\x00")))
        off += len(idx) + 5
        footer = meta_h + idx_h
        footer += b"\x00" * (40 - len(footer))
        f.write(footer + struct.pack("<Q", TABLE_MAGIC))


def _read_varint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        if not c & 0x80:
            return v, i
        s += 7


def _read_block(raw: bytes, off: int, size: int, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    data = raw[off: off + size]
    if verify:
        (crc,) = struct.unpack("<I", raw[off + size + 1: off + size + 5])
        if crc != _mcrc(data + raw[off + size: off + size + 1]):
            raise IOError("SSTable block CRC mismatch")
    (nr,) = struct.unpack("<I", data[-4:])
    end = len(data) - 4 - 4 * nr
    out, i, last = [], 0, b""
    while i < end:
        shared, i = _read_varint(data, i)
        nonshared, i = _read_varint(data, i)
        vlen, i = _read_varint(data, i)
        key = last[:shared] + data[i: i + nonshared]
        i += nonshared
        out.append((key, data[i: i + vlen]))
        i += vlen
        last = key
    return out


def read_sstable(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    raw = open(path, "rb").read()
    (magic,) = struct.unpack("<Q", raw[-8:])
    if magic != TABLE_MAGIC:
        raise IOError("not an SSTable (bad magic)")
    footer = raw[-48:-8]
    i = 0
    _, i = _read_varint(footer, i)
    _, i = _read_varint(footer, i)
    ioff, i = _read_varint(footer, i)
    isz, i = _read_varint(footer, i)
    out = []
    for _, h in _read_block(raw, ioff, isz, verify):
        j = 0
        boff, j = _read_varint(h, j)
        bsz, j = _read_varint(h, j)
        out += _read_block(raw, boff, bsz, verify)
    return out


# ------------------------------------------------------------------------------ bundle API
def _as_numpy(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        t = t.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().contiguous().numpy()
    return np.ascontiguousarray(t)


def write_bundle(prefix: str, tensors: Dict[str, object], chunk_bytes: int = 1 << 28) -> None:
    """Write ``prefix.index`` + ``prefix.data-00000-of-00001`` (TF tensor_bundle V2)."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    entries = []
    off = 0
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        for name in sorted(tensors):
            t = tensors[name]
            if isinstance(t, torch.Tensor) and t.numel() * t.element_size() > chunk_bytes and t.dim() >= 1:
                # stream huge tables chunk by chunk (e.g. the 882M-row fm_v): CRC32C is chained
                rows = max(1, chunk_bytes // max(1, t[0].numel() * 4))
                crc, size, dt = 0, 0, None
                for r0 in range(0, t.shape[0], rows):
                    a = _as_numpy(t[r0: r0 + rows])
                    dt = _NP2DT[a.dtype]
                    b = a.tobytes()
                    f.write(b)
                    crc = _nio.crc32c_extend(crc, b)
                    size += len(b)
                entries.append((name.encode(), bundle_entry(dt, tuple(t.shape), off, size,
                                                            _nio.mask_crc(crc))))
                off += size
                continue
            a = _as_numpy(t)
            b = a.tobytes()
            f.write(b)
            entries.append((name.encode(), bundle_entry(_NP2DT[a.dtype], a.shape, off, len(b), _mcrc(b))))
            off += len(b)
    entries.append((b"", bundle_header(1)))
    write_sstable(prefix + ".index", entries)


def data_path(prefix: str, shard: int, num_shards: int) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def parse_header(b: bytes) -> dict:
    d = {"num_shards": 1}
    for f, _, v in _fields(b):
        if f == 1:
            d["num_shards"] = v
    return d


class ShardWriter:
    """One data shard ``prefix.data-<shard>-of-<num>`` of a multi-shard bundle.  ``add`` streams a
    tensor (or an iterator of row chunks of it) into the shard and returns its index entry; the
    entries of every shard go to ``write_index`` (one writer, e.g. rank 0).  Each rank writes only
    its own shard -- no host ever holds the whole checkpoint."""

    def __init__(self, prefix: str, shard: int, num_shards: int):
        os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
        self.shard, self.num = shard, num_shards
        self.f = open(data_path(prefix, shard, num_shards), "wb")
        self.off = 0
        self.entries: List[Tuple[bytes, bytes]] = []

    def add(self, name: str, shape: Tuple[int, ...], chunks: Iterable) -> Tuple[bytes, bytes]:
        crc, size, dt = 0, 0, None
        for c in chunks:
            a = _as_numpy(c)
            dt = _NP2DT[a.dtype]
            b = a.tobytes()
            self.f.write(b)
            crc = _nio.crc32c_extend(crc, b)
            size += len(b)
        e = (name.encode(), bundle_entry(dt, tuple(int(x) for x in shape), self.off, size,
                                         _nio.mask_crc(crc), shard_id=self.shard))
        self.off += size
        self.entries.append(e)
        return e

    def close(self):
        self.f.close()


def write_index(prefix: str, entries: List[Tuple[bytes, bytes]], num_shards: int) -> None:
    write_sstable(prefix + ".index", list(entries) + [(b"", bundle_header(num_shards))])


def read_bundle(prefix: str, verify: bool = True, names: Optional[Iterable[str]] = None
                ) -> Dict[str, np.ndarray]:
    items = read_sstable(prefix + ".index", verify)
    want = set(names) if names is not None else None
    num = 1
    for k, v in items:
        if not k:
            num = parse_header(v)["num_shards"]
    out = {}
    files = {}
    try:
        for k, v in items:
            if not k:
                continue
            name = k.decode()
            if want is not None and name not in want:
                continue
            e = parse_entry(v)
            sid = e["shard_id"]
            if sid not in files:
                files[sid] = open(data_path(prefix, sid, num), "rb")
            f = files[sid]
            f.seek(e["offset"])
            b = f.read(e["size"])
            if verify and len(b) < (1 << 26) and _mcrc(b) != e["crc32c"]:
                raise IOError(f"tensor {name}: data CRC mismatch")
            out[name] = np.frombuffer(b, dtype=_DT2NP[e["dtype"]]).reshape(e["shape"]).copy()
    finally:
        for f in files.values():
            f.close()
    return out


def write_checkpoint_state(model_dir: str, latest: str, all_paths: List[str]) -> None:
    """The ``checkpoint`` text proto Estimator uses to find the latest checkpoint."""
    lines = [f'model_checkpoint_path: "{latest}"'] + [f'all_model_checkpoint_paths: "{p}"' for p in all_paths]
    tmp = os.path.join(model_dir, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(model_dir, "checkpoint"))


def read_checkpoint_state(model_dir: str) -> Optional[str]:
    p = os.path.join(model_dir, "checkpoint")
    if not os.path.exists(p):
        return None
    for line in open(p):
        if line.startswith("model_checkpoint_path:"):
            return line.split(":", 1)[1].strip().strip('"')
    return None
