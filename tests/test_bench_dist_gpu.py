"""The N>1 path of bench.py, run end to end before the driver's scaling runs do: `python bench.py --gpus 2` re-runs
itself under torch.distributed.run (spawn_ranks), each rank builds the model and the ZeRO-1 engine, warms up, times
its steps between barriers, and the ranks' seconds are gathered and reduced by MAX (reference launcher:
scripts/spatialvla_4b_pretrain/torchrun_pretrain.sh:48-89, train/dist_utils.py:41-46).  The test box has one GPU, so
both ranks share cuda:0 over gloo (--share-device --backend gloo); the 8-GPU run takes the same code with one rank per
GPU over RCCL.  Asserted: exactly one JSON line (rank 0), n_gpus 2, global_batch 2 x B, and value / ms_per_step
computed from the MAX of the per-rank seconds."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(420)
@pytest.mark.parametrize("world", [2, 8])
def test_bench_ranks_one_json_line(cuda, world):
    """world 2, and world 8 = configs[3]'s rank count (ZeRO-1 chunks of 8 x 64-element padded buckets)."""
    B, steps, warmup = 2, 2, 1
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(world), "--config", "tiny", "--batch", str(B),
           "--steps", str(steps), "--warmup", str(warmup), "--backend", "gloo", "--share-device",
           "--no-cpu-baseline", "--no-decode", "--no-fp8-leg"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == world
    assert r["config"]["global_batch"] == world * B and r["config"]["per_gpu_batch"] == B
    assert r["config"]["parallelism"] == f"dp{world}" and r["scaling"] == "weak" and r["backend"] == "gloo"
    per = r["per_rank_seconds"]
    assert len(per) == world and all(t > 0 for t in per)
    assert r["timed_seconds_max"] == pytest.approx(max(per), rel=1e-6)
    assert r["ms_per_step"] == pytest.approx(max(per) / steps * 1e3, rel=1e-3, abs=0.01)
    assert r["value"] == pytest.approx(world * B * steps / max(per), rel=1e-3)
    assert r["roofline"]["launches_timed"] > 0
    assert r["final_loss"] == r["final_loss"]  # not NaN
