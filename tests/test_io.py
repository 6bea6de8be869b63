"""I/O tests: TFRecord framing + CRC, Example codec, libsvm, native loader,
shard policy coverage (disjoint + complete: fixes quirk Q1)."""
import os
import random
import struct

import numpy as np
import pytest
import torch

import hipfm
from hipfm.data import native_io as nio
from hipfm.data import tfrecord as tr
from hipfm.data.pipeline import InputPipeline, discover_files, plan_shard, shard_spec


def _rows(n, F, seed=0):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, 1 << 40, size=(n, F), dtype=np.int64)
    vals = rng.random((n, F), dtype=np.float32)
    lab = (rng.random(n) < 0.3).astype(np.float32)
    return lab, ids, vals


def test_crc32c_known_vectors():
    # RFC 3720 test vector: 32 bytes of zeros -> 0x8a9136aa
    assert tr.crc32c(b"\x00" * 32) == 0x8A9136AA
    assert nio.crc32c(b"\x00" * 32) == 0x8A9136AA
    assert tr.crc32c(b"123456789") == 0xE3069283
    data = bytes(range(256)) * 7
    assert nio.crc32c(data) == tr.crc32c(data)
    assert nio.masked_crc32c(data) == tr.masked_crc32c(data)


def test_example_roundtrip_python_and_native():
    F = 39
    lab, ids, vals = _rows(3, F)
    for i in range(3):
        b = tr.encode_example(lab[i], ids[i].tolist(), vals[i].tolist())
        l2, i2, v2 = tr.parse_deepfm_example(b, F)
        assert l2 == lab[i] and i2 == ids[i].tolist()
        assert np.allclose(v2, vals[i])
        l3, i3, v3 = nio.decode_example(b, F)
        assert l3 == lab[i] and np.array_equal(i3, ids[i]) and np.array_equal(v3, vals[i])
    with pytest.raises(ValueError):
        nio.decode_example(tr.encode_example(1.0, [1, 2], [1.0, 2.0]), F)


def test_example_decoder_accepts_unpacked_and_reordered_fields():
    # hand-built Example with unpacked int64/float lists and the features in another order
    def ld(f, p):
        return tr._key(f, 2) + tr._varint(len(p)) + p
    ids_list = b"".join(tr._key(1, 0) + tr._varint(v) for v in (5, 7))
    vals_list = b"".join(tr._key(1, 5) + struct.pack("<f", v) for v in (0.5, 2.0))
    lab_list = tr._key(1, 5) + struct.pack("<f", 1.0)
    feats = [("values", ld(2, vals_list)), ("label", ld(2, lab_list)), ("ids", ld(3, ids_list))]
    entries = b"".join(ld(1, ld(1, k.encode()) + ld(2, v)) for k, v in feats)
    ex = ld(1, entries)
    lab, ids, vals = nio.decode_example(ex, 2)
    assert lab == 1.0 and ids.tolist() == [5, 7] and vals.tolist() == [0.5, 2.0]
    assert tr.parse_deepfm_example(ex, 2) == (1.0, [5, 7], [0.5, 2.0])


def test_tfrecord_file_roundtrip_and_crc_detection(tmp_path):
    F = 5
    lab, ids, vals = _rows(100, F, 1)
    p = str(tmp_path / "tr-0.tfrecords")
    nio.write_examples(p, lab, ids, vals)
    # python reader verifies every CRC of the native writer's output
    recs = list(tr.read_records(p))
    assert len(recs) == 100
    assert tr.parse_deepfm_example(recs[7], F)[1] == ids[7].tolist()
    assert nio.count_records(p) == 100
    # corrupt one payload byte -> CRC error from both readers
    raw = bytearray(open(p, "rb").read())
    raw[40] ^= 0xFF
    q = str(tmp_path / "bad.tfrecords")
    open(q, "wb").write(raw)
    with pytest.raises(IOError):
        list(tr.read_records(q))
    with pytest.raises(IOError):
        list(nio.NativeLoader([q], F, 10))


def test_libsvm_parse_and_convert(tmp_path):
    src = tmp_path / "train.libsvm"
    src.write_text("1 1:0.5 2:0.03519 3:1\n0 4:1 5:0.25 9:2\n\n")
    assert tr.parse_libsvm_line("1 1:0.5 2:0.03519 3:1") == (1.0, [1, 2, 3], [0.5, 0.03519, 1.0])
    n = nio.libsvm_to_tfrecord(str(src), str(tmp_path / "a.tfrecords"), 3)
    assert n == 2
    n2 = tr.libsvm_to_tfrecord(str(src), str(tmp_path / "b.tfrecords"), 3)
    assert n2 == 2
    assert open(tmp_path / "a.tfrecords", "rb").read() == open(tmp_path / "b.tfrecords", "rb").read()
    batches = list(nio.NativeLoader([str(src)], 3, 2, fmt=nio.FMT_LIBSVM))
    assert len(batches) == 1
    lab, ids, vals = batches[0]
    assert lab.tolist() == [1.0, 0.0] and ids[1].tolist() == [4, 5, 9]


@pytest.mark.parametrize("threads", [1, 3])
def test_native_loader_batches_deterministic(tmp_path, threads):
    F = 4
    files = []
    allrows = []
    for k in range(5):
        lab, ids, vals = _rows(700 + 13 * k, F, k)
        p = str(tmp_path / f"tr-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
        allrows.append(ids)
    b1 = [x[1].copy() for x in nio.NativeLoader(files, F, 256, threads=threads)]
    b2 = [x[1].copy() for x in nio.NativeLoader(files, F, 256, threads=threads)]
    assert len(b1) == len(b2) and all(np.array_equal(a, b) for a, b in zip(b1, b2))
    total = sum(len(r) for r in allrows)
    assert len(b1) == total // 256                       # drop_remainder=True
    got = np.concatenate(b1)
    want = np.concatenate(allrows)
    assert set(map(tuple, got.tolist())) <= set(map(tuple, want.tolist()))
    # no drop: every record exactly once
    full = np.concatenate([x[1] for x in nio.NativeLoader(files, F, 256, drop_remainder=False,
                                                          threads=threads)])
    assert sorted(map(tuple, full.tolist())) == sorted(map(tuple, want.tolist()))


@pytest.mark.parametrize("threads,drop", [(1, True), (3, True), (3, False)])
def test_compact_values_are_lossless(tmp_path, threads, drop):
    """Compact wire format (hfm_io.cpp Loader::next with a value mask): a batch ships only the
    value columns of fields that are not all exactly 1.0 in its chunks; expanding them back gives
    the plain batch bit for bit.  Fields: always 1.0 (categorical, never shipped), real-valued
    (always shipped), 1.0 except in one record of one file (shipped only in the batches that
    touch that record's chunk), and -0.0 / NaN patterns (not 1.0: shipped)."""
    F = 7
    files = []
    for k in range(4):
        lab, ids, _ = _rows(900 + 37 * k, F, k)
        ids = ids % 100_000
        vals = np.ones(ids.shape, np.float32)
        vals[:, 1] = np.random.default_rng(k).standard_normal(len(ids)).astype(np.float32)
        vals[:, 4] = np.where(np.arange(len(ids)) % 5 == 0, 0.5, 1.0)
        if k == 2:
            vals[300, 5] = 2.0
        if k == 3:
            vals[10, 6] = -0.0
            vals[11, 6] = np.nan
        p = str(tmp_path / f"c-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    B = 256
    plain = nio.NativeLoader(files, F, B, threads=threads, drop_remainder=drop, ids32=True)
    comp = nio.NativeLoader(files, F, B, threads=threads, drop_remainder=drop, ids32=True)
    masks = []
    while True:
        lab0, ids0, val0 = (np.empty(B, np.float32), np.empty((B, F), np.int32), np.empty((B, F), np.float32))
        r0 = plain.next_into(lab0, ids0, val0)
        lab1, ids1, vc = np.empty(B, np.float32), np.empty((B, F), np.int32), np.empty(B * F, np.float32)
        r1, mask = comp.next_into_compact(lab1, ids1, vc)
        assert r0 == r1
        if r0 == 0:
            break
        masks.append(mask)
        assert mask & 0b11 == 0b10                       # field 0 never shipped, field 1 always
        assert np.array_equal(lab0[:r0], lab1[:r0]) and np.array_equal(ids0[:r0], ids1[:r0])
        full = nio.expand_values(vc, r0, F, mask)
        assert np.array_equal(full.view(np.uint32), val0[:r0].view(np.uint32))
        # a field left out is exactly 1.0 in every row of the batch
        for f in range(F):
            if not (mask >> f) & 1:
                assert (val0[:r0, f].view(np.uint32) == np.float32(1.0).view(np.uint32)).all()
    assert any(m >> 5 & 1 for m in masks) and not all(m >> 5 & 1 for m in masks)
    assert any(m >> 6 & 1 for m in masks)
    plain.close()
    comp.close()


@pytest.mark.parametrize("compact,threads", [(False, 1), (True, 3)])
def test_assembly_ring_matches_next_into(tmp_path, compact, threads):
    """hfm_io.cpp Loader::start_ring: an assembler thread fills registered buffers ahead of the
    consumer in cyclic slot order; ring_take returns the same batches, in the same order, as
    next_into (values compact or not), whatever order the consumer holds and hands slots back in.
    A loader destroyed while its assembler waits for a slot, and a bad id, end cleanly."""
    F, B = 5, 128
    files = []
    for k in range(3):
        lab, ids, vals = _rows(700 + 41 * k, F, k)
        ids = ids % 50_000
        vals[:, 0] = 1.0
        p = str(tmp_path / f"a-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    want = []
    ld = nio.NativeLoader(files, F, B, threads=threads, drop_remainder=False, ids32=True)
    while True:
        bl, bi, bv = np.empty(B, np.float32), np.empty((B, F), np.int32), np.empty((B, F), np.float32)
        r = ld.next_into(bl, bi, bv)
        if r == 0:
            break
        want.append((bl[:r].copy(), bi[:r].copy(), bv[:r].copy()))
    ld.close()
    n = 4
    bufs = [(np.empty(B, np.float32), np.empty((B, F), np.int32), np.empty(B * F, np.float32)) for _ in range(n)]
    ld = nio.NativeLoader(files, F, B, threads=threads, drop_remainder=False, ids32=True)
    ld.start_ring(bufs, compact=compact)
    got, held = [], []
    while True:
        r, slot, mask = ld.ring_take()
        if r == 0:
            break
        bl, bi, bv = bufs[slot]
        vals = nio.expand_values(bv, r, F, mask) if compact else bv[:r * F].reshape(r, F)
        if compact:
            assert not mask & 1                       # field 0 is all 1.0: never shipped
        got.append((bl[:r].copy(), bi[:r].copy(), vals.copy()))
        held.append(slot)
        if len(held) == n - 1:                     # hand back the oldest two (out of take order)
            ld.ring_give(held.pop(1))
            ld.ring_give(held.pop(0))
    for s in held:
        ld.ring_give(s)
    assert ld.ring_take()[0] == 0                  # the end stays the end
    ld.close()
    assert len(got) == len(want)
    for (a1, a2, a3), (b1, b2, b3) in zip(got, want):
        assert np.array_equal(a1, b1) and np.array_equal(a2, b2)
        assert np.array_equal(a3.view(np.uint32), b3.view(np.uint32))
    # destroyed while the assembler waits for a slot (every slot taken, none given back)
    ld = nio.NativeLoader(files, F, B, threads=threads, ids32=True)
    ld.start_ring(bufs[:2], compact=compact)
    ld.ring_take()
    ld.ring_take()
    ld.close()
    # a decode error reaches the taker
    ld = nio.NativeLoader(files, F, B, threads=threads, ids32=True, id_limit=10)
    ld.start_ring(bufs[:2], compact=compact)
    with pytest.raises(IOError, match="outside"):
        for _ in range(20):
            r, slot, _ = ld.ring_take()
            ld.ring_give(slot)
    ld.close()


def test_record_shard_matches_reference_semantics(tmp_path):
    F = 3
    lab, ids, vals = _rows(50, F, 9)
    p = str(tmp_path / "tr.tfrecords")
    nio.write_examples(p, lab, ids, vals)
    for n in (2, 3):
        for i in range(n):
            got = np.concatenate([x[1] for x in nio.NativeLoader([p], F, 1, record_shard=(n, i))])
            assert np.array_equal(got, ids[i::n])


def test_shard_plan_disjoint_and_complete():
    files = [f"f{i}" for i in range(11)]
    for n in (1, 2, 3, 8):
        seen = []
        for i in range(n):
            plan = plan_shard(files, n, i, "file", seed=3, epoch=2)
            assert plan.record_shard == (1, 0) or n == 1
            seen += plan.files
        assert sorted(seen) == sorted(files)            # disjoint + complete
    # fewer files than ranks -> record-level shard of the identical order
    p0 = plan_shard(files[:2], 4, 1, "file", seed=3)
    assert p0.record_shard == (4, 1) and sorted(p0.files) == files[:2]


def test_shard_spec_matrix():
    assert shard_spec(8, 5, 1, 4, 2, enable_s3_shard=False) == (8, 5)
    assert shard_spec(8, 5, 1, 4, 2, enable_s3_shard=True) == (4, 1)
    assert shard_spec(8, 5, 1, 4, 2, pipe_mode=True, enable_data_multi_path=True) == (2, 1)
    assert shard_spec(8, 5, 1, 4, 2, pipe_mode=True, enable_data_multi_path=True,
                      enable_s3_shard=True) == (1, 0)
    assert shard_spec(8, 5, 1, 4, 2, pipe_mode=True, enable_s3_shard=True) == (4, 1)


def test_discover_and_pipeline_cache(tmp_path):
    F = 3
    d = tmp_path / "data" / "sub"
    d.mkdir(parents=True)
    for k in range(3):
        lab, ids, vals = _rows(100, F, k)
        nio.write_examples(str(d / f"tr-{k}.tfrecords"), lab, ids, vals)
    nio.write_examples(str(d / "va-0.tfrecords"), *_rows(10, F, 7))
    tr_files = discover_files(str(tmp_path / "data"), "tr")
    assert len(tr_files) == 3 and len(discover_files(str(tmp_path / "data"), "va")) == 1
    pipe = InputPipeline(tr_files, F, 64, num_epochs=2, cache=True, seed=1)
    e0 = [b[0] for b in pipe.iter_epoch(0)]
    e1 = [b[0] for b in pipe.iter_epoch(1)]
    assert len(e0) == 300 // 64 and all(torch.equal(a, b) for a, b in zip(e0, e1))
    assert pipe.local_records() == 300


@pytest.mark.parametrize("fmt", ["tfrecord", "libsvm"])
def test_loader_rejects_ids_outside_vocabulary(tmp_path, fmt):
    """An id >= feature_size (or negative) fails the read with the file and record named, before
    anything reaches the device (whose gathers / row updates index the table unchecked)."""
    F, V = 3, 1000
    lab, ids, vals = _rows(40, F, 5)
    ids = ids % V
    ids[17, 2] = V + 3                                  # corrupted record 17
    if fmt == "tfrecord":
        p = str(tmp_path / "tr-0.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        kind = nio.FMT_TFRECORD
    else:
        p = str(tmp_path / "tr-0.txt")
        with open(p, "w") as f:
            for i in range(len(lab)):
                f.write(f"{lab[i]:g} " + " ".join(f"{ids[i, j]}:{vals[i, j]:g}" for j in range(F)) + "\n")
        kind = nio.FMT_LIBSVM
    ok = [x for x in nio.NativeLoader([p], F, 8, fmt=kind)]          # unchecked: reads through
    assert len(ok) == 5
    with pytest.raises(IOError, match=r"feature id 1003 \(field 2\).*feature_size=1000.*record 17"):
        list(nio.NativeLoader([p], F, 8, fmt=kind, id_limit=V))
    pipe = InputPipeline([p], F, 8, fmt=fmt, id_limit=V)
    with pytest.raises(IOError, match="tr-0"):
        list(pipe.iter_epoch(0))
    ids[17, 2] = 5
    if fmt == "tfrecord":
        nio.write_examples(p, lab, ids, vals)
        assert len(list(nio.NativeLoader([p], F, 8, fmt=kind, id_limit=V))) == 5


@pytest.mark.parametrize("threads,drop,ring", [(1, True, False), (3, False, False), (3, True, True)])
def test_raw_loader_ships_the_records_of_the_decoding_loader(tmp_path, threads, drop, ring):
    """Raw mode (hfm_io.cpp Loader::next_raw, the GPU-decode wire): each batch carries the records'
    serialized Examples back to back + B + 1 offsets, in exactly the order the decoding loader
    returns its rows; decoding the shipped bytes on the host gives the decoded batches bit for bit
    (the GPU decoder, csrc/kernels/decode.hip, is checked against them in tests/test_gpu_decode.py)."""
    F, B = 6, 128
    files = []
    for k in range(4):
        lab, ids, vals = _rows(300 + 17 * k, F, 30 + k)
        p = str(tmp_path / f"tr-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    ref = [(a.copy(), b.copy(), c.copy()) for a, b, c in
           nio.NativeLoader(files, F, B, threads=threads, drop_remainder=drop)]
    ld = nio.NativeLoader(files, F, B, threads=threads, drop_remainder=drop, raw=True)
    bufs = [(torch.zeros(B * 1024, dtype=torch.uint8), torch.zeros(B + 1, dtype=torch.int32)) for _ in range(3)]
    got = []
    if ring:
        ld.start_ring_raw(bufs)
    while True:
        if ring:
            r, slot, nb = ld.ring_take()
            raw, offs = bufs[slot]
        else:
            raw, offs = bufs[0]
            r, nb = ld.next_raw_into(raw, offs)
        if r == 0:
            break
        o = offs.numpy().astype(np.int64)
        assert o[0] == 0 and o[r] == nb
        rows = [nio.decode_example(raw.numpy()[o[i]:o[i + 1]].tobytes(), F) for i in range(r)]
        got.append((np.array([x[0] for x in rows], np.float32), np.stack([x[1] for x in rows]),
                    np.stack([x[2] for x in rows])))
        if ring:
            ld.ring_give(slot)
    ld.close()
    assert len(got) == len(ref)
    for (l1, i1, v1), (l2, i2, v2) in zip(got, ref):
        assert np.array_equal(l1, l2) and np.array_equal(i1, i2) and np.array_equal(v1, v2)


@pytest.mark.parametrize("threads", [1, 3])
def test_raw_loader_device_crc_ships_each_records_data_crc(tmp_path, threads):
    """device_crc (verify mode 2): the workers check only the length CRCs and append each record's
    stored masked data CRC to its bytes (the GPU decoder verifies it); a corrupted payload byte
    reaches the batch unflagged by the host -- with the stored CRC that exposes it."""
    F, B = 6, 64
    files = []
    for k in range(2):
        lab, ids, vals = _rows(150 + 9 * k, F, 50 + k)
        p = str(tmp_path / f"tr-{k}.tfrecords")
        nio.write_examples(p, lab, ids, vals)
        files.append(p)
    plain = nio.NativeLoader(files, F, B, threads=threads, raw=True)
    dev = nio.NativeLoader(files, F, B, threads=threads, raw=True, device_crc=True)
    assert dev.device_crc and not plain.device_crc
    bufs = [(torch.zeros(B * 1024, dtype=torch.uint8), torch.zeros(B + 1, dtype=torch.int32)) for _ in range(2)]
    nb_all = 0
    while True:
        r1, n1 = plain.next_raw_into(*bufs[0])
        r2, n2 = dev.next_raw_into(*bufs[1])
        assert r1 == r2
        if r1 == 0:
            break
        assert n2 == n1 + 4 * r1
        o1, o2 = bufs[0][1].numpy().astype(np.int64), bufs[1][1].numpy().astype(np.int64)
        for i in range(r1):
            rec = bufs[0][0].numpy()[o1[i]:o1[i + 1]].tobytes()
            got = bufs[1][0].numpy()[o2[i]:o2[i + 1]].tobytes()
            assert got[:-4] == rec
            assert int.from_bytes(got[-4:], "little") == nio.masked_crc32c(rec)
        nb_all += r1
    plain.close()
    dev.close()
    assert nb_all > 0
    # one payload byte flipped in the first record: the host-CRC loader refuses the file, the
    # device-CRC loader ships it (with the stored CRC, which no longer matches)
    raw = bytearray(open(files[0], "rb").read())
    raw[12 + 5] ^= 0x40
    bad = str(tmp_path / "bad.tfrecords")
    open(bad, "wb").write(bytes(raw))
    ld = nio.NativeLoader([bad], F, B, threads=1, raw=True)
    with pytest.raises(IOError, match="data CRC"):
        ld.next_raw_into(*bufs[0])
    ld.close()
    ld = nio.NativeLoader([bad], F, B, threads=1, raw=True, device_crc=True)
    r, nb = ld.next_raw_into(*bufs[1])
    assert r == B
    o = bufs[1][1].numpy().astype(np.int64)
    first = bufs[1][0].numpy()[o[0]:o[1]].tobytes()
    assert int.from_bytes(first[-4:], "little") != nio.masked_crc32c(first[:-4])
    ld.close()


def test_raw_loader_reports_a_batch_larger_than_its_buffer(tmp_path):
    F = 6
    lab, ids, vals = _rows(300, F, 3)
    p = str(tmp_path / "tr-0.tfrecords")
    nio.write_examples(p, lab, ids, vals)
    ld = nio.NativeLoader([p], F, 128, threads=1, raw=True)
    with pytest.raises(IOError, match="exceeds"):
        ld.next_raw_into(torch.zeros(1000, dtype=torch.uint8), torch.zeros(129, dtype=torch.int32))
    ld.close()
