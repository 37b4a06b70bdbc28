set -o pipefail
export TMPDIR=/tmp
TAG=r8l AB_TESTS="tests/test_decode_gpu.py" tools/ab.sh decode 2 "-" "SVLA_DECODE_PREFETCH=2" "SVLA_DECODE_PREFETCH=3" "SVLA_DECODE_PREFETCH=3 SVLA_DECODE_PREFETCH_BLOCKS=256"
