"""The GPU decoder's parallel CRC32C (csrc/kernels/decode.hip payload_crc), emulated on the CPU:
8 equal segments after front zero-padding, slice-by-8 steps, the first 4 bytes inverted for the
initial register, a 3-level combine by x^(8 seg 2^l) mod P -- equal to the plain CRC32C
(data/tfrecord.py, TF's record_writer masking) for every length class the kernel takes."""
import numpy as np
import pytest

from hipfm.data import tfrecord as tr

POLY = 0x82F63B78


def _x1(b):
    return (b >> 1) ^ POLY if b & 1 else b >> 1


def _mulmod(a, b):
    p = 0
    for k in range(32):
        if a & (0x80000000 >> k):
            p ^= b
        b = _x1(b)
    return p


def _tables():
    t0 = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = _x1(c)
        t0.append(c)
    T = [t0]
    for k in range(1, 8):
        T.append([(T[k - 1][i] >> 8) ^ t0[T[k - 1][i] & 0xFF] for i in range(256)])
    return T


T = _tables()


def _ops(seg):
    x = 0x80000000
    for _ in range(8 * seg):
        x = _x1(x)
    o1 = x
    o2 = _mulmod(o1, o1)
    return o1, o2, _mulmod(o2, o2)


def _segmented_crc(msg: bytes) -> int:
    n = len(msg)
    assert 64 <= n <= 8 * 8 * 128
    seg = ((n + 63) // 64) * 8
    z = 8 * seg - n

    def byte(i):
        return msg[i] ^ (0xFF if i < 4 else 0)
    v = []
    for lane in range(8):
        b1 = (lane + 1) * seg - z
        pos = max(lane * seg - z, 0)
        c = 0
        while pos < b1 and (b1 - pos) & 7:
            c = T[0][(c ^ byte(pos)) & 0xFF] ^ (c >> 8)
            pos += 1
        while pos < b1:
            lo = byte(pos) | byte(pos + 1) << 8 | byte(pos + 2) << 16 | byte(pos + 3) << 24
            hi = byte(pos + 4) | byte(pos + 5) << 8 | byte(pos + 6) << 16 | byte(pos + 7) << 24
            c ^= lo
            c = (T[7][c & 0xFF] ^ T[6][(c >> 8) & 0xFF] ^ T[5][(c >> 16) & 0xFF] ^ T[4][c >> 24] ^
                 T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24])
            pos += 8
        v.append(c)
    ops = _ops(seg)
    for lvl in range(3):
        step = 1 << lvl
        for i in range(0, 8, 2 * step):
            v[i] = _mulmod(ops[lvl], v[i]) ^ v[i + step]
    return (~v[0]) & 0xFFFFFFFF


@pytest.mark.parametrize("n", [64, 65, 71, 72, 100, 127, 128, 129, 300, 511, 1000, 1024, 4097, 8192])
def test_segmented_crc_equals_crc32c(n):
    msg = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8).tobytes()
    assert _segmented_crc(msg) == tr.crc32c(msg)


def test_segmented_crc_of_an_example_record():
    ex = tr.encode_example(1.0, list(range(39)), [0.5] * 39)
    assert len(ex) >= 64
    c = _segmented_crc(ex)
    masked = (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF
    assert masked == tr.masked_crc32c(ex)
