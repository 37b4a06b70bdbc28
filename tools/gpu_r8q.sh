set -o pipefail
export TMPDIR=/tmp
TAG=r8q tools/ab.sh step 2 "SVLA_SIDE_CU_RESERVE=0" "SVLA_SIDE_CU_RESERVE=16" "SVLA_SIDE_CU_RESERVE=8"
