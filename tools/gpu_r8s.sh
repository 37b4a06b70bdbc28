set -o pipefail
export TMPDIR=/tmp
TAG=r8s2 tools/ab.sh step 2 "SVLA_SIDE_CU_RESERVE=8" "SVLA_SIDE_CU_RESERVE=4" "SVLA_SIDE_CU_RESERVE=2"
