# Kernel-trace a short bench run and print the steady-state step breakdown (tools/summarize_profile.py).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-pk}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode > gpurun_out/$TAG/bench_prof.json 2> gpurun_out/$TAG/bench_prof.err && \
python tools/summarize_profile.py trace /tmp/prof_$TAG gpurun_out/$TAG/$TAG > gpurun_out/$TAG/trace_summary.log 2>&1
