# GPU parity tests, then the headline bench 3x
set -o pipefail
bash tools/gpu_tests.sh || exit 1
bash tools/gpu_ab.sh
