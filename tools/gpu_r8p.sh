set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/beit_gemm_bench.py 2>&1 | grep -v amdgpu.ids
