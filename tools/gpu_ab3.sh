#!/bin/bash
set -o pipefail
bash tools/sweep.sh && bash tools/stats2.sh
