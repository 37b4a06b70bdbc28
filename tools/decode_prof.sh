# Kernel-trace the decode benchmark (graph replays) and summarise the steady-state decode steps.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-decprof}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pd_$TAG -o dec --output-format csv -- python3 tools/decode_bench.py --reps 1 --long 60 --no-uncached > $O/decode_prof.json 2> $O/decode_prof.err && \
cp $(find /tmp/pd_$TAG -name "*kernel_stats.csv" | head -1) $O/${TAG}_kernel_stats.csv && \
python3 tools/decode_trace_summary.py /tmp/pd_$TAG > $O/${TAG}_step_breakdown.txt
