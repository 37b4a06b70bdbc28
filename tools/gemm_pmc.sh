# SQ counters of the 8-phase GEMM on one shape (gemm_bench.py "gate/up fwd"), one counter set per pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gpmc
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d /tmp/gp$i -o pmc --output-format csv -- python3 tools/gemm_bench.py "gate/up fwd" "gate/up dgrad" > $O/run$i.log 2>&1 || exit 1
  f=$(find /tmp/gp$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" > $O/pmc$i.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"][:60] + " grid=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "gemm" not in k:
        continue
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()}, "n=", len(next(iter(d.values()))))
PY
done
ls $O
