set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ckpt_diag.py 2>&1 | grep -v Warning | tail -45
