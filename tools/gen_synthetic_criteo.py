#!/usr/bin/env python
"""Write a synthetic Criteo-shaped dataset (libsvm and/or TFRecord) with learnable labels.

  python tools/gen_synthetic_criteo.py --out /tmp/criteo --preset reference --train_rows 100000 \
      --val_rows 10000 --files 4 [--format tfrecord|libsvm|both]

Files follow the reference naming (PS:374-377): tr-*.tfrecords, va-*.tfrecords, te-*.tfrecords.
See hipfm/data/synthetic.py for the distribution (Zipf ids, hidden teacher labels).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_libsvm(path, lab, ids, vals):
    with open(path, "w") as f:
        for i in range(len(lab)):
            f.write("%g " % lab[i] + " ".join("%d:%g" % (a, b) for a, b in zip(ids[i], vals[i])) + "\n")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--preset", default="reference")
    ap.add_argument("--train_rows", type=int, default=100000)
    ap.add_argument("--val_rows", type=int, default=10000)
    ap.add_argument("--test_rows", type=int, default=0)
    ap.add_argument("--files", type=int, default=4, help="train files")
    ap.add_argument("--format", default="tfrecord", choices=["tfrecord", "libsvm", "both"])
    ap.add_argument("--seed", type=int, default=2024)
    a = ap.parse_args(argv)
    import hipfm  # noqa: F401
    from hipfm.data.native_io import write_examples
    from hipfm.data.synthetic import make_synth
    g = make_synth(a.preset, seed=a.seed)
    os.makedirs(a.out, exist_ok=True)
    step = 0

    def emit(prefix, rows, nfiles):
        nonlocal step
        per = (rows + nfiles - 1) // max(1, nfiles)
        left = rows
        for k in range(nfiles):
            n = min(per, left)
            if n <= 0:
                break
            ids, vals, lab = g.batch(n, step=step)
            step += 1
            ids, vals, lab = ids.numpy(), vals.numpy(), lab.numpy()
            if a.format in ("tfrecord", "both"):
                write_examples(os.path.join(a.out, f"{prefix}-{k}.tfrecords"), lab, ids, vals)
            if a.format in ("libsvm", "both"):
                write_libsvm(os.path.join(a.out, f"{prefix}-{k}.libsvm"), lab, ids, vals)
            left -= n

    emit("tr", a.train_rows, a.files)
    emit("va", a.val_rows, 1)
    if a.test_rows:
        emit("te", a.test_rows, 1)
    print(f"feature_size={g.feature_size} field_size={g.F} -> {a.out}")


if __name__ == "__main__":
    main()
