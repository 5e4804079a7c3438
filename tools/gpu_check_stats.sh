bash tools/gpu_check.sh && bash tools/stats2.sh
