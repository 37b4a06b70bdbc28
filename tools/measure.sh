# Measurement on one MI355X: bench line, rocprofv3 kernel-trace/stats, PMC HBM traffic passes.
# Raw rocprof output is condensed on the box (tools/summarize_profile.py) and then deleted.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode > $O/bench_prof.json 2> $O/bench_prof.err && \
python tools/summarize_profile.py trace /tmp/prof_$TAG $O/$TAG > $O/trace_summary.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
python tools/summarize_profile.py pmc /tmp/pmc_fetch $O/${TAG}_pmc_fetch > $O/pmc_fetch_summary.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode > $O/pmc_write.json 2> $O/pmc_write.err && \
python tools/summarize_profile.py pmc /tmp/pmc_write $O/${TAG}_pmc_write > $O/pmc_write_summary.log 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/blk_$TAG -o blk --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/block.log 2>&1 && \
python tools/block_trace.py /tmp/blk_$TAG > $O/${TAG}_block_breakdown.txt 2>&1
rc=$?
ls -la $O
exit $rc
