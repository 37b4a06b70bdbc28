"""Host-side (Python) cost of one Gemma2 layer fwd+bwd, bf16 vs fp8 projections: cProfile over 10 iterations of
tools/block_ab.py's workload, top functions by total time."""
import cProfile, os, pstats, sys, io
sys.argv = [sys.argv[0], "1", "1", "3"]
mode = os.environ.get("SVLA_BLOCK_FP8")
import runpy
pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "block_ab.py"), run_name="__main__")
except SystemExit:
    pass
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
