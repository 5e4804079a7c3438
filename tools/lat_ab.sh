#!/bin/bash
# the latency-path switches one at a time (tools/lat_ab.py per setting)
set -o pipefail
timeout -k 10 120 python tools/lat_ab.py default || exit 1
MPG_OWN_STREAM=0 timeout -k 10 120 python tools/lat_ab.py no_own_stream || exit 1
MPG_SMALL_HOST_SC=0 timeout -k 10 120 python tools/lat_ab.py no_host_sc || exit 1
MPG_OWN_STREAM=0 MPG_SMALL_HOST_SC=0 timeout -k 10 120 python tools/lat_ab.py round3_like || exit 1
