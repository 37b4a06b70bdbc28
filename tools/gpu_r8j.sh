set -o pipefail
export TMPDIR=/tmp
TAG=r8j2 tools/ab.sh decode 2 "SVLA_LIB=diag/libsvla_dpre1.so" "SVLA_LIB=diag/libsvla_dpre2.so" "SVLA_LIB=diag/libsvla_dpre3.so"
