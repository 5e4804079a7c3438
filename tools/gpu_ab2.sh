#!/bin/bash
# variant timings with and without the two-stream overlap
set -o pipefail
bash tools/sweep.sh && bash tools/sweep.sh MPG_OVERLAP_MIN=1000000000000
