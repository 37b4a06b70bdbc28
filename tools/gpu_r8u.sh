set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/block_ab.py flag wgrad_split 4 2>&1 | grep -v amdgpu.ids || exit 1
TAG=r8u tools/ab.sh step 2 "SVLA_WGRAD_SPLIT=0" "SVLA_WGRAD_SPLIT=1"
