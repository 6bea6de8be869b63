#!/usr/bin/env python
"""libsvm -> TFRecord converter (reference C36, tools/libsvm_to_tfrecord.py).

The reference hard-codes its input/output paths and uses a TF1 InteractiveSession (Q12); this
is a proper CLI over the native C++ converter (csrc/io, same Example schema: label FloatList[1],
ids Int64List[F], values FloatList[F]):

  python tools/libsvm_to_tfrecord.py --field_size 39 train.libsvm tr.tfrecords [va.libsvm va.tfrecords ...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--field_size", type=int, required=True, help="F: id:val pairs per line")
    ap.add_argument("--python", action="store_true", help="use the pure-Python writer")
    ap.add_argument("pairs", nargs="+", help="src dst [src dst ...]")
    a = ap.parse_args(argv)
    if len(a.pairs) % 2:
        ap.error("arguments must be (src, dst) pairs")
    import hipfm  # noqa: F401
    from hipfm.data import native_io, tfrecord
    for src, dst in zip(a.pairs[::2], a.pairs[1::2]):
        n = (tfrecord.libsvm_to_tfrecord(src, dst, a.field_size) if a.python
             else native_io.libsvm_to_tfrecord(src, dst, a.field_size))
        print(f"{src} -> {dst}: {n} records")


if __name__ == "__main__":
    main()
