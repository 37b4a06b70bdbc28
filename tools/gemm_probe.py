"""Ad-hoc GEMM shapes through tools/gemm_bench.run: python tools/gemm_probe.py MxNxK:lay ... (lay nt|nn|tn);
SVLA_VARIANTS=0,3 compares dispatch variants in one process (hipBLASLt as the yardstick)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_bench import run

for spec in sys.argv[1:]:
    dims, lay = spec.split(":")
    m, n, k = (int(v) for v in dims.split("x"))
    run(spec, m, n, k, lay)
