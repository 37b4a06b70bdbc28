set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6o}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_g -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
python tools/summarize_profile.py trace /tmp/prof_g $O/${TAG:-r6o} > $O/trace_summary.log 2>&1
head -20 $O/${TAG:-r6o}_step_breakdown.txt
