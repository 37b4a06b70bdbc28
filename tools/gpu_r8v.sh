set -o pipefail
export TMPDIR=/tmp
TAG=r8v bash tools/measure.sh
