#!/bin/bash
# BVH-mesh contacts + the rest of the mesh suite on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mesh.py tests/test_gpu_parity.py -m gpu -k "mesh or contact" -x -v --timeout 300 --timeout-method thread > gpurun_out/mesh_ct.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/mesh_ct.log | head -60
tail -3 gpurun_out/mesh_ct.log
exit $rc
