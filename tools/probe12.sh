set -o pipefail
mkdir -p gpurun_out/probe12
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/probe12/t.txt 2>&1; rc=$?
tail -3 gpurun_out/probe12/t.txt
exit $rc
