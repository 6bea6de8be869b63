"""TFRecord framing + ``tf.train.Example`` codec, pure Python (no TensorFlow needed).

Reference contract (``tools/libsvm_to_tfrecord.py:25-32`` and the parse spec
``PS:81-86``): one Example per sample with

    label  : FloatList[1]
    ids    : Int64List[F]
    values : FloatList[F]

TFRecord framing (TF ``io/record_writer.cc`` format): ``uint64 length | uint32 masked_crc32c(length)
| data | uint32 masked_crc32c(data)``, little endian, masked_crc = ((crc >> 15) | (crc << 17)) +
0xa282ead8.

This module is the reference implementation used by the converter tool and the tests; the
fast path (threaded reader, CRC32C with SSE4.2, zero-copy decode into batch buffers) is the
C++ library ``csrc/io`` bound in ``data/native_io.py``.
"""
from __future__ import annotations

import struct
from typing import BinaryIO, Iterable, Iterator, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------- CRC32C
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------- framing
def write_record(f: BinaryIO, data: bytes) -> None:
    hdr = struct.pack("<Q", len(data))
    f.write(hdr)
    f.write(struct.pack("<I", masked_crc32c(hdr)))
    f.write(data)
    f.write(struct.pack("<I", masked_crc32c(data)))


def iter_records(f: BinaryIO, verify: bool = True) -> Iterator[bytes]:
    while True:
        hdr = f.read(8)
        if not hdr:
            return
        if len(hdr) < 8:
            raise IOError("truncated TFRecord header")
        (n,) = struct.unpack("<Q", hdr)
        (hcrc,) = struct.unpack("<I", f.read(4))
        if verify and hcrc != masked_crc32c(hdr):
            raise IOError("TFRecord length CRC mismatch")
        data = f.read(n)
        if len(data) < n:
            raise IOError("truncated TFRecord payload")
        (dcrc,) = struct.unpack("<I", f.read(4))
        if verify and dcrc != masked_crc32c(data):
            raise IOError("TFRecord data CRC mismatch")
        yield data


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        yield from iter_records(f, verify)


class TFRecordWriter:
    def __init__(self, path: str):
        self.f = open(path, "wb")

    def write(self, data: bytes):
        write_record(self.f, data)

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---------------------------------------------------------------------------- protobuf wire
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _float_list(vals: Sequence[float]) -> bytes:       # FloatList { repeated float value = 1 [packed] }
    return _ld(1, struct.pack(f"<{len(vals)}f", *vals))


def _int64_list(vals: Sequence[int]) -> bytes:         # Int64List { repeated int64 value = 1 [packed] }
    return _ld(1, b"".join(_varint(int(v)) for v in vals))


def _feature(kind: int, payload: bytes) -> bytes:      # Feature { oneof: bytes=1 float=2 int64=3 }
    return _ld(kind, payload)


def encode_example(label: float, ids: Sequence[int], values: Sequence[float]) -> bytes:
    """Serialize ``tf.train.Example{label, ids, values}`` exactly as CONV:25-32 builds it."""
    feats = [("label", _feature(2, _float_list([float(label)]))),
             ("ids", _feature(3, _int64_list(ids))),
             ("values", _feature(2, _float_list(values)))]
    entries = b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, v)) for k, v in feats)
    return _ld(1, entries)   # Example { Features features = 1 } ; Features { map<...> feature = 1 }


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = 0
    v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _fields(b: bytes):
    i, n = 0, len(b)
    while i < n:
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
            yield f, wt, v
        elif wt == 1:
            yield f, wt, b[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _read_varint(b, i)
            yield f, wt, b[i:i + ln]
            i += ln
        elif wt == 5:
            yield f, wt, b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _decode_feature(b: bytes):
    for kind, wt, payload in _fields(b):
        if kind == 2:      # FloatList
            out: List[float] = []
            for f, w, v in _fields(payload):
                if w == 2:
                    out.extend(struct.unpack(f"<{len(v) // 4}f", v))
                elif w == 5:
                    out.append(struct.unpack("<f", v)[0])
            return out
        if kind == 3:      # Int64List
            out2: List[int] = []
            for f, w, v in _fields(payload):
                if w == 2:
                    j = 0
                    while j < len(v):
                        x, j = _read_varint(v, j)
                        out2.append(x - (1 << 64) if x >= (1 << 63) else x)
                elif w == 0:
                    out2.append(v - (1 << 64) if v >= (1 << 63) else v)
            return out2
        if kind == 1:
            return [v for f, w, v in _fields(payload)]
    return []


def decode_example(b: bytes) -> dict:
    """Parse a serialized Example into {feature name: list of values} (any field order)."""
    feats = {}
    for f, wt, features in _fields(b):
        if f != 1:
            continue
        for f2, wt2, entry in _fields(features):
            if f2 != 1:
                continue
            key, val = None, b""
            for f3, wt3, v in _fields(entry):
                if f3 == 1:
                    key = v.decode()
                elif f3 == 2:
                    val = v
            if key is not None:
                feats[key] = _decode_feature(val)
    return feats


def parse_deepfm_example(b: bytes, field_size: int) -> Tuple[float, List[int], List[float]]:
    """FixedLenFeature parse (PS:81-86): label [], ids [F], values [F] — errors on wrong F."""
    d = decode_example(b)
    label = d.get("label", [])
    ids = d.get("ids", [])
    vals = d.get("values", [])
    if len(label) != 1 or len(ids) != field_size or len(vals) != field_size:
        raise ValueError(f"Example does not match the fixed schema (F={field_size}): "
                         f"label {len(label)}, ids {len(ids)}, values {len(vals)}")
    return float(label[0]), [int(x) for x in ids], [float(x) for x in vals]


# ---------------------------------------------------------------------------- libsvm
def parse_libsvm_line(line: str) -> Tuple[float, List[int], List[float]]:
    """``label id:val id:val ...`` (CONV:15-23)."""
    parts = line.split()
    if not parts:
        raise ValueError("empty libsvm line")
    label = float(parts[0])
    ids, vals = [], []
    for tok in parts[1:]:
        i, _, v = tok.partition(":")
        ids.append(int(i))
        vals.append(float(v))
    return label, ids, vals


def libsvm_to_tfrecord(src: str, dst: str, field_size: Optional[int] = None) -> int:
    """Convert a libsvm file to TFRecord Examples; returns the record count."""
    n = 0
    with open(src) as fi, TFRecordWriter(dst) as w:
        for line in fi:
            if not line.strip():
                continue
            label, ids, vals = parse_libsvm_line(line)
            if field_size is not None and len(ids) != field_size:
                raise ValueError(f"line {n + 1}: {len(ids)} features, expected {field_size}")
            w.write(encode_example(label, ids, vals))
            n += 1
    return n
