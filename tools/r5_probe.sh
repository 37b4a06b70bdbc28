#!/bin/bash
# Round-5 probe call: gemm4 k-loop stamps with ablations, MFMA-busy PMC of the isolated Gemma2 block (every kernel in
# situ), attention PMC, the bench line and the block trace.  Each GPU step has its own time limit; a crash or timeout
# stops the script.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
TAG=${TAG:-r5a}
O=$R/gpurun_out/$TAG
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -gt 1 ]; then echo "[$name] stopping: crash or timeout"; exit $rc; fi
  return 0
}
if [ -n "$TESTS" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -k "$TESTS" ${PYX--x} -v -s --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1
  tail -5 $O/pytest.txt
  mkdir -p $O/parity && cp gpurun_out/parity/*.json $O/parity/ 2>/dev/null
fi
if [ -n "$BLOCK_AB" ]; then
  step block_ab 300 python -u tools/block_lib_ab.py spatialvla_amd/libsvla.so $BLOCK_AB 5 > $O/block_ab.txt 2>&1
  cat $O/block_ab.txt
fi
if [ -n "$BLOCK_FLAG" ]; then
  step block_flag 300 python -u tools/block_ab.py flag $BLOCK_FLAG 6 > $O/block_flag.txt 2>&1
  cat $O/block_flag.txt
fi
if [ -n "$TRACE_AB" ]; then  # in-situ block breakdown for the main library and for $TRACE_AB
  step trace_a 180 rocprofv3 --kernel-trace --stats -d /tmp/tra -o t --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/trace_a.log 2>&1
  python tools/block_trace.py /tmp/tra > $O/block_breakdown_main.txt 2>&1
  export SVLA_LIB=$R/$TRACE_AB
  step trace_b 180 rocprofv3 --kernel-trace --stats -d /tmp/trb -o t --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/trace_b.log 2>&1
  unset SVLA_LIB
  python tools/block_trace.py /tmp/trb > $O/block_breakdown_alt.txt 2>&1
  paste $O/block_breakdown_main.txt $O/block_breakdown_alt.txt | cut -c1-200
fi
if [ -n "$MXDBG" ]; then
  step mxdbg 120 python -u tools/mx_debug.py > $O/mx_debug.txt 2>&1
  cat $O/mx_debug.txt
fi
if [ -n "$LIST" ]; then timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; fi
if [ -n "$STAMPS" ]; then
  step stamps 300 python -u tools/stamps_multi.py $STAMPS -- $STAMP_SHAPES > $O/stamps.txt 2>&1
  cat $O/stamps.txt
fi
if [ -n "$AB_LIB" ]; then
  step gemm_ab 300 python -u tools/gemm_ab.py spatialvla_amd/libsvla.so $AB_LIB $AB_SHAPES > $O/gemm_ab.txt 2>&1
  cat $O/gemm_ab.txt
fi
if [ -n "$BLOCK_PMC" ]; then
  step blk_pmc1 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d /tmp/bp1 -o p1 --output-format csv -- python3 tools/block_ab.py 1 1 3 > $O/blk_pmc1.log 2>&1
  step blk_pmc2 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d /tmp/bp2 -o p2 --output-format csv -- python3 tools/block_ab.py 1 1 3 > $O/blk_pmc2.log 2>&1
  step blk_trace 180 rocprofv3 --kernel-trace --stats -d /tmp/bt -o bt --output-format csv -- python3 tools/block_ab.py 1 1 5 > $O/blk_trace.log 2>&1
  python tools/block_trace.py /tmp/bt > $O/block_breakdown.txt 2>&1
  cp /tmp/bt/*/*kernel_stats.csv $O/blk_kernel_stats.csv 2>/dev/null
  python tools/pmc_dispatch.py /tmp/bp1 /tmp/bp2 > $O/block_pmc.txt 2>&1
  mkdir -p $O/bp1 $O/bp2 && cp $(find /tmp/bp1 -name "*counter_collection.csv") $O/bp1/ && cp $(find /tmp/bp2 -name "*counter_collection.csv") $O/bp2/
  cat $O/block_breakdown.txt
fi
if [ -n "$GEMM_PMC" ]; then
  for shp in $GEMM_PMC; do
    step gemm_pmc 400 tools/gemm_pmc2.sh $TAG ${shp//,/ } > $O/gemm_pmc_$shp.log 2>&1
  done
  for f in $O/*_svla.txt $O/*_torch.txt; do echo "== $f"; cat $f; done
fi
if [ -n "$FP8_PMC" ]; then
  for arm in $FP8_PMC; do
    step fp8_run 120 python3 tools/fp8_pmc_one.py $arm 9984 18432 2304 20 >> $O/fp8_runs.txt 2>&1
    step fp8_pmc1 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d /tmp/f8p1_$arm -o p1 --output-format csv -- python3 tools/fp8_pmc_one.py $arm 9984 18432 2304 10 > /dev/null 2>&1
    step fp8_pmc2 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d /tmp/f8p2_$arm -o p2 --output-format csv -- python3 tools/fp8_pmc_one.py $arm 9984 18432 2304 10 > /dev/null 2>&1
    python tools/pmc_table.py /tmp/f8p1_$arm /tmp/f8p2_$arm > $O/fp8_pmc_$arm.txt 2>&1
  done
  cat $O/fp8_runs.txt; grep -A16 "gemm4" $O/fp8_pmc_*.txt
fi
if [ -n "$ATT_PMC" ]; then
  for spec in $ATT_PMC; do  # e.g. gemma2:fwd gemma2:bwd beit:fwd
    shp=${spec%%:*}; what=${spec##*:}; d=/tmp/att_${shp}_${what}
    step att_trace 120 rocprofv3 --kernel-trace --stats -d ${d}_t -o t --output-format csv -- python3 tools/attn_one.py $shp $what 10 > /dev/null 2>&1
    step att_pmc1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d ${d}_1 -o p1 --output-format csv -- python3 tools/attn_one.py $shp $what 10 > /dev/null 2>&1
    step att_pmc2 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d ${d}_2 -o p2 --output-format csv -- python3 tools/attn_one.py $shp $what 10 > /dev/null 2>&1
    python tools/pmc_table.py ${d}_t ${d}_1 ${d}_2 > $O/attn_pmc_${shp}_${what}.txt 2>&1
    cat $O/attn_pmc_${shp}_${what}.txt
  done
fi
if [ -n "$NORM_AB" ]; then
  step norm_ab 300 python -u tools/norm_ab.py spatialvla_amd/libsvla.so $NORM_AB > $O/norm_ab.txt 2>&1
  cat $O/norm_ab.txt
fi
if [ -n "$GEGLU_AB" ]; then
  step geglu_ab 300 python -u tools/geglu_ab.py $GEGLU_AB > $O/geglu_ab.txt 2>&1
  cat $O/geglu_ab.txt
fi
if [ -n "$GEMM_BENCH" ]; then
  step gemm_bench 400 python -u tools/gemm_bench.py > $O/gemm_bench.txt 2>&1
  cat $O/gemm_bench.txt
fi
if [ -n "$AB_ENV" ]; then
  step ab_env 1100 tools/ab_env.sh $AB_ENV ${AB_ROUNDS:-2} $AB_VALS > $O/ab_env.txt 2>&1
  cat $O/ab_env.txt
fi
if [ -n "$BENCH" ]; then
  step bench 600 python -u bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err
  head -c 2500 $O/bench.json; echo
fi
ls $O
