set -o pipefail
bash tools/sweep.sh && bash tools/kt.sh nowalk MPG_DEBUG_NO_WALK=1 > /tmp/kt2.out 2>&1 && grep -E "==|narrow|cull" /tmp/kt2.out && bash tools/stats2.sh
