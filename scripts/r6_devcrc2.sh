#!/bin/bash
# round 6: GPU data CRC vs host CRC, streamed epochs + host-only raw ingest passes; decode kernel time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARMS="1 2" bash scripts/stream_decode_ab.sh 16000000 64 3 --epochs 3 || exit 1
