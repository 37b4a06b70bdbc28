set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/zoe_cost.py 5 2>&1 | grep -v Warning | tail -5
