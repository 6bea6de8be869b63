#!/bin/bash
# Host-side ingest probe on the GPU box's CPUs: decode microbenchmark + loader thread sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=/tmp/hipfm_io_$$
timeout -k 10 300 python tools/gen_synthetic_criteo.py --out "$D" --preset criteo_kaggle \
  --train_rows 2000000 --val_rows 16384 --files 16 > gpurun_out/io_datagen.log 2>&1 || { echo datagen failed; exit 1; }
g++ -O3 -std=c++17 -msse4.2 -pthread tools/io_microbench.cpp -o /tmp/io_microbench_$$ && \
  timeout -k 10 120 /tmp/io_microbench_$$ $(ls $D/tr* | head -1)
echo "nproc $(nproc); $(grep -m1 'model name' /proc/cpuinfo)"
timeout -k 10 300 python tools/ingest_sweep.py "$D"
rm -rf "$D" /tmp/io_microbench_$$
