set -o pipefail
export TMPDIR=/tmp
TAG=r8x tools/ab.sh decode 2 "-" "SVLA_GEMM_VARIANT=7"
