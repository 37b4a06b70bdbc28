set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe9
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pf9 -o pf --output-format csv -- python3 tools/decode_bench.py --reps 3 --long 4 --new-tokens 1 --no-uncached > gpurun_out/probe9/dec.json 2> gpurun_out/probe9/dec.err || exit 1
python3 tools/prefill_trace_summary.py /tmp/pf9 > gpurun_out/probe9/prefill_breakdown.txt 2>&1
