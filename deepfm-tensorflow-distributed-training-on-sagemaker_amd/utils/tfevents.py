"""TensorBoard event files without TensorFlow (the reference's Estimator writes
``loss``, ``global_step/sec`` summaries to ``model_dir`` and eval metrics to ``model_dir/eval``
through its default hooks; PS:432-435, HVD:365-368, DOC p.34 shows those log lines).

File format: ``events.out.tfevents.<time>.<host>`` holds TFRecord-framed (masked CRC32C)
``tensorflow.Event`` protos.  Only the fields TensorBoard needs for scalars are encoded, by hand:

  Event   { double wall_time = 1; int64 step = 2; string file_version = 3; Summary summary = 5; }
  Summary { repeated Value value = 1; }
  Value   { string tag = 1; float simple_value = 2; }
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Iterator, Optional, Tuple

from ..data.tfrecord import iter_records, write_record


def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, scalars: Optional[Dict[str, float]] = None,
                 file_version: Optional[str] = None) -> bytes:
    out = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        out += _len_field(3, file_version.encode())
    if scalars:
        summ = b"".join(_len_field(1, _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v)))
                        for tag, v in scalars.items())
        out += _len_field(5, summ)
    return out


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    n = s = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return n, i


def decode_event(b: bytes) -> dict:
    """Inverse of encode_event for the encoded fields (tests / tools)."""
    ev = {"scalars": {}}
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 1:
            ev["wall_time"] = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif w == 0:
            v, i = _read_varint(b, i)
            if f == 2:
                ev["step"] = v
        elif w == 2:
            n, i = _read_varint(b, i)
            p = b[i:i + n]
            i += n
            if f == 3:
                ev["file_version"] = p.decode()
            elif f == 5:
                j = 0
                while j < len(p):
                    _, j = _read_varint(p, j)
                    m, j = _read_varint(p, j)
                    val, j = p[j:j + m], j + m
                    tag, sv, q = None, None, 0
                    while q < len(val):
                        kk, q = _read_varint(val, q)
                        if kk >> 3 == 1:
                            mm, q = _read_varint(val, q)
                            tag, q = val[q:q + mm].decode(), q + mm
                        elif kk & 7 == 5:
                            sv, q = struct.unpack_from("<f", val, q)[0], q + 4
                    ev["scalars"][tag] = sv
        elif w == 5:
            i += 4
    return ev


class EventFileWriter:
    """Append-only scalar event file in ``logdir`` (created on first use)."""

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self.f = open(self.path, "ab")
        write_record(self.f, encode_event(time.time(), 0, file_version="brain.Event:2"))
        self.f.flush()

    def scalars(self, step: int, values: Dict[str, float]):
        write_record(self.f, encode_event(time.time(), step, values))
        self.f.flush()

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None


def read_events(path: str) -> Iterator[dict]:
    with open(path, "rb") as f:
        for rec in iter_records(f):
            yield decode_event(rec)
