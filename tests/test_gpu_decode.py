"""GPU decode of serialized tf.train.Example records (csrc/kernels/decode.hip) against the host
decoder (csrc/io/hfm_io.cpp decode_example): the raw loader's batches decoded on the device equal
the decoding loader's batches bit for bit; malformed records and out-of-vocabulary ids are flagged
(never a fault, never garbage ids); hand-built Examples with unpacked lists and reordered
features decode like TF's parser would."""
import struct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data import native_io as nio  # noqa: E402
from hipfm.data import tfrecord as tr  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402

DEV = torch.device("cuda", 0)


def _rows(n, F, seed, big=False):
    rng = np.random.default_rng(seed)
    hi = (1 << 31) - 1 if big else 1 << 20
    ids = rng.integers(0, hi, size=(n, F), dtype=np.int64)
    vals = rng.random((n, F), dtype=np.float32)
    vals[:, F // 2:] = 1.0
    lab = (rng.random(n) < 0.3).astype(np.float32)
    return lab, ids, vals


def _decode(raw: bytes, offs, F, limit=0, crc=False):
    rows = len(offs) - 1
    draw = torch.tensor(list(raw) or [0], dtype=torch.uint8, device=DEV)
    doffs = torch.tensor(offs, dtype=torch.int64).to(torch.int32).to(DEV)
    ids = torch.full((rows, F), -7, dtype=torch.int32, device=DEV)
    vals = torch.full((rows, F), -7.0, device=DEV)
    lab = torch.full((rows,), -7.0, device=DEV)
    err = torch.tensor([0, 0x7FFFFFFF], dtype=torch.int32, device=DEV)
    KN.decode_examples(draw, doffs, rows, F, limit, ids, vals, lab, err, crc=crc)
    torch.cuda.synchronize()
    return ids.cpu(), vals.cpu(), lab.cpu(), err.tolist()


@pytest.mark.parametrize("F,big,dcrc", [(39, True, False), (39, False, False), (100, True, False), (3, False, False),
                                         (39, True, True), (100, True, True), (3, False, True), (1, False, True)])
def test_gpu_decode_matches_the_host_decoder(tmp_path, F, big, dcrc):
    B = 256
    files = []
    for k in range(3):
        lab, ids, vals = _rows(500 + 11 * k, F, 40 + k, big)
        p = str(tmp_path / f"tr-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    ref = [(a.copy(), b.copy(), c.copy()) for a, b, c in nio.NativeLoader(files, F, B, threads=2, ids32=True)]
    # dcrc: records carry their data CRCs, verified by the decoder (short records at F = 1, 3 take
    # its one-lane path, longer ones the 8-segment path)
    ld = nio.NativeLoader(files, F, B, threads=2, raw=True, device_crc=dcrc)
    raw = torch.zeros(B * 2048, dtype=torch.uint8, pin_memory=True)
    offs = torch.zeros(B + 1, dtype=torch.int32, pin_memory=True)
    n = 0
    while True:
        r, nb = ld.next_raw_into(raw, offs)
        if r == 0:
            break
        ids, vals, lab, err = _decode(bytes(raw[:nb].numpy()), offs[:r + 1].tolist(), F, crc=dcrc)
        l2, i2, v2 = ref[n]
        assert err == [0, 0x7FFFFFFF]
        assert torch.equal(ids, torch.from_numpy(i2)) and torch.equal(vals, torch.from_numpy(v2))
        assert torch.equal(lab, torch.from_numpy(l2))
        n += 1
    ld.close()
    assert n == len(ref)


def test_gpu_decode_unpacked_and_reordered_example():
    def ld(f, p):
        return tr._key(f, 2) + tr._varint(len(p)) + p
    ids_list = b"".join(tr._key(1, 0) + tr._varint(v) for v in (5, 300, 2 ** 31 - 1))
    vals_list = b"".join(tr._key(1, 5) + struct.pack("<f", v) for v in (0.5, 2.0, -1.0))
    lab_list = tr._key(1, 5) + struct.pack("<f", 1.0)
    feats = [("values", ld(2, vals_list)), ("extra", ld(1, ld(1, b"xyz"))), ("label", ld(2, lab_list)),
             ("ids", ld(3, ids_list))]
    ex = ld(1, b"".join(ld(1, ld(1, k.encode()) + ld(2, v)) for k, v in feats))
    packed = tr.encode_example(0.0, [1, 2, 3], [1.0, 1.0, 4.0])
    ids, vals, lab, err = _decode(ex + packed, [0, len(ex), len(ex) + len(packed)], 3)
    assert err == [0, 0x7FFFFFFF]
    assert ids.tolist() == [[5, 300, 2 ** 31 - 1], [1, 2, 3]]
    assert vals.tolist() == [[0.5, 2.0, -1.0], [1.0, 1.0, 4.0]] and lab.tolist() == [1.0, 0.0]


def test_gpu_decode_flags_bad_records_without_faulting():
    F = 4
    good = tr.encode_example(1.0, [1, 2, 3, 4], [0.5, 1.0, 1.0, 1.0])
    short = tr.encode_example(1.0, [1, 2, 3], [0.5, 1.0, 1.0])            # F - 1 values
    oov = tr.encode_example(0.0, [1, 2, 999, 4], [1.0, 1.0, 1.0, 1.0])     # id >= limit
    trunc = good[:-5]                                                      # cut inside the values
    recs = [good, short, good, oov, trunc, good]
    offs = np.cumsum([0] + [len(r) for r in recs]).tolist()
    ids, vals, lab, err = _decode(b"".join(recs), offs, F, limit=100)
    assert err[0] == 3 and err[1] == 1                                    # schema + id bits, first bad row 1
    for i in (0, 2, 5):
        assert ids[i].tolist() == [1, 2, 3, 4] and lab[i].item() == 1.0
    for i in (1, 4):                                                       # zeroed rows
        assert ids[i].tolist() == [0] * F and vals[i].tolist() == [0.0] * F and lab[i].item() == 0.0
    assert ids[3].tolist() == [1, 2, 0, 4]                                 # the bad id written as 0


@pytest.mark.parametrize("nbytes_pad", [0, 700, 9000])
def test_gpu_decode_flags_a_corrupt_record_by_its_crc(nbytes_pad):
    """crc mode: every record's masked CRC32C checked on the GPU (one-lane path for short records,
    8 segments + combine up to 8 KB, one lane again beyond); a flipped payload byte or a wrong
    stored CRC zeroes that row only and reports bit value 4 with the smallest bad index."""
    F = 39
    lab, ids, vals = _rows(12, F, 77)
    recs = []
    for i in range(12):
        ex = tr.encode_example(float(lab[i]), [int(x) for x in ids[i]], [float(v) for v in vals[i]])
        if nbytes_pad:      # an unknown top-level field (bytes) pads the record: skipped by the parser
            ex = ex + tr._key(9, 2) + tr._varint(nbytes_pad) + bytes(range(256)) * (nbytes_pad // 256) + \
                bytes(nbytes_pad % 256)
        recs.append(bytearray(ex + struct.pack("<I", tr.masked_crc32c(ex))))
    good = b"".join(bytes(r) for r in recs)
    offs = [0]
    for r in recs:
        offs.append(offs[-1] + len(r))
    i0, v0, l0, e0 = _decode(good, offs, F, crc=True)
    assert e0 == [0, 0x7FFFFFFF]
    assert torch.equal(i0, torch.from_numpy(ids.astype(np.int32))) and torch.equal(l0, torch.from_numpy(lab))
    recs[5][len(recs[5]) // 2] ^= 0x10          # payload byte of record 5
    recs[9][-1] ^= 0x01                          # stored CRC of record 9
    i1, v1, l1, e1 = _decode(b"".join(bytes(r) for r in recs), offs, F, crc=True)
    assert e1 == [4, 5]
    for k in (5, 9):
        assert not i1[k].any() and not v1[k].any() and l1[k] == 0
    keep = [k for k in range(12) if k not in (5, 9)]
    assert torch.equal(i1[keep], i0[keep]) and torch.equal(v1[keep], v0[keep])
