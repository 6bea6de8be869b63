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


def _decode(raw: bytes, offs, F, limit=0):
    rows = len(offs) - 1
    draw = torch.tensor(list(raw) or [0], dtype=torch.uint8, device=DEV)
    doffs = torch.tensor(offs, dtype=torch.int64).to(torch.int32).to(DEV)
    ids = torch.full((rows, F), -7, dtype=torch.int32, device=DEV)
    vals = torch.full((rows, F), -7.0, device=DEV)
    lab = torch.full((rows,), -7.0, device=DEV)
    err = torch.tensor([0, 0x7FFFFFFF], dtype=torch.int32, device=DEV)
    KN.decode_examples(draw, doffs, rows, F, limit, ids, vals, lab, err)
    torch.cuda.synchronize()
    return ids.cpu(), vals.cpu(), lab.cpu(), err.tolist()


@pytest.mark.parametrize("F,big", [(39, True), (39, False), (100, True), (3, False)])
def test_gpu_decode_matches_the_host_decoder(tmp_path, F, big):
    B = 256
    files = []
    for k in range(3):
        lab, ids, vals = _rows(500 + 11 * k, F, 40 + k, big)
        p = str(tmp_path / f"tr-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    ref = [(a.copy(), b.copy(), c.copy()) for a, b, c in nio.NativeLoader(files, F, B, threads=2, ids32=True)]
    ld = nio.NativeLoader(files, F, B, threads=2, raw=True)
    raw = torch.zeros(B * 2048, dtype=torch.uint8, pin_memory=True)
    offs = torch.zeros(B + 1, dtype=torch.int32, pin_memory=True)
    n = 0
    while True:
        r, nb = ld.next_raw_into(raw, offs)
        if r == 0:
            break
        ids, vals, lab, err = _decode(bytes(raw[:nb].numpy()), offs[:r + 1].tolist(), F)
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
