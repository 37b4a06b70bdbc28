#!/bin/bash
# Final-measurement call B: a rocprofv3 kernel trace of the training step, the HBM PMC passes of the dominant kernel
# (FETCH_SIZE and WRITE_SIZE in separate runs) and the isolated Gemma2 block breakdown.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r5}
O=gpurun_out/$TAG
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -gt 1 ]; then echo "[$name] stopping: crash or timeout"; exit $rc; fi
  return 0
}
step trace 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > $O/bench_prof.json 2> $O/bench_prof.err
python tools/summarize_profile.py trace /tmp/prof_$TAG $O/$TAG > $O/trace_summary.log 2>&1
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > $O/pmc_fetch.json 2> $O/pmc_fetch.err
python tools/summarize_profile.py pmc /tmp/pmc_fetch $O/${TAG}_pmc_fetch > $O/pmc_fetch_summary.log 2>&1
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode --no-fp8-leg > $O/pmc_write.json 2> $O/pmc_write.err
python tools/summarize_profile.py pmc /tmp/pmc_write $O/${TAG}_pmc_write > $O/pmc_write_summary.log 2>&1
step block 300 rocprofv3 --kernel-trace -d /tmp/blk_$TAG -o blk --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/block.log 2>&1
python tools/block_trace.py /tmp/blk_$TAG > $O/${TAG}_block_breakdown.txt 2>&1
ls -la $O
