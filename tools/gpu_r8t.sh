set -o pipefail
export TMPDIR=/tmp
TAG=r8t bash tools/trace.sh block
