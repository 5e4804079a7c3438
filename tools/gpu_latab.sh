#!/bin/bash
# latency-path split with the MPG_DIAG library (variants/diag): full, FK + sphere
# test only (7), no narrow test (3); then the bare launch/sync floors
set -o pipefail
for m in 0 7 3; do
  LD_LIBRARY_PATH=$PWD/variants/diag MPG_DEBUG_CULL=$m timeout -k 10 120 python tools/lat_ablate.py || exit 1
done
timeout -k 10 120 python tools/latency.py || exit 1
