"""GPU: bench.py's multi-rank path on hardware (VERDICT r05 "Next round" 1).

`bench.py --gpus 2` spawns two fresh rank processes (127.0.0.1 rendezvous, gloo group); each rank picks its device as
LOCAL_RANK modulo the devices it sees, so on a one-GPU lease both ranks run on device 0 -- the per-rank contexts, the
once-per-device block-table probe, per-rank ceilings and the gathered per-rank fields all execute on the GPU, which
is the only hardware evidence for BASELINE's 2/4/8-GPU axis a one-GPU box can give (the 8-GPU scaling runs are the
driver's).  Both workloads: config2 (objects per rank, weak scaling) and config5 (a fixed job split over the ranks,
strong scaling), reduced in size so each run takes well under a minute.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, timeout=300):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)  # bench.py spawns its own ranks
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 prints the one line
    return json.loads(lines[0])


def device_count():
    import torch

    return torch.cuda.device_count()  # counts without initialising the runtime in this process


def check_common(line, n=2):
    assert line["n_gpus"] == n
    assert line["world_size_initialised"] == n
    assert line["process_group_backend"] == "gloo"
    assert line["verified_per_rank"] == [True] * n
    assert line["breakdown"]["verified"] is True
    assert len(line["kernel_ms_per_rank"]) == n and all(v > 0 for v in line["kernel_ms_per_rank"])
    assert len(line["decode_ms_per_rank"]) == n and all(v > 0 for v in line["decode_ms_per_rank"])
    assert line["device_per_rank"] == [r % device_count() for r in range(n)]
    assert line["value"] > 0 and line["ms_per_step"] > 0


@pytest.mark.timeout(400)
def test_two_ranks_config2_weak():
    objs = 4
    line = run_bench(["--gpus", "2", "--objects", str(objs), "--steps", "3", "--warmup", "1", "--breakdown-steps", "4",
                      "--no-cpu-baseline", "--no-ceiling"])
    check_common(line)
    assert line["scaling"] == "weak"
    assert line["config"]["objects_per_gpu"] == objs
    assert line["config"]["objects_total"] == 2 * objs  # every rank ran its own objects
    k, L, n = 32, 1 << 20, 64
    per_rank = objs * (n * (k * L + k + L) + k * (k + L))
    assert line["value"] == pytest.approx(2 * per_rank * 3 / (line["ms_per_step"] * 3e-3) / (1 << 30), rel=2e-3)


@pytest.mark.timeout(400)
def test_two_ranks_config5_strong_split():
    job = 33  # odd: rank 0 takes 17, rank 1 takes 16
    line = run_bench(["--gpus", "2", "--workload", "config5", "--objects", str(job), "--chunk", "8", "--steps", "2",
                      "--warmup", "1", "--breakdown-steps", "2", "--no-cpu-baseline", "--no-ceiling"])
    check_common(line)
    assert line["scaling"] == "strong"
    assert line["config"]["objects_total"] == job  # the split covers every object of the fixed job exactly once
    assert line["config"]["objects_per_gpu"] == job // 2 + 1  # rank 0's share
    assert line["config"]["objects_per_launch"] == 8


@pytest.mark.timeout(400)
def test_four_ranks_config5_strong_split():
    """Four ranks on the lease's GPU (profiles/r06_config5_n4_onegpu.json is the full job the same way): the ragged
    split (35 = 9 + 9 + 9 + 8) covers the job once and every rank verifies its share."""
    job = 35
    line = run_bench(["--gpus", "4", "--workload", "config5", "--objects", str(job), "--chunk", "8", "--steps", "2",
                      "--warmup", "1", "--breakdown-steps", "2", "--no-cpu-baseline", "--no-ceiling"])
    check_common(line, n=4)
    assert line["scaling"] == "strong"
    assert line["config"]["objects_total"] == job
    assert line["config"]["objects_per_gpu"] == job // 4 + 1  # rank 0's share
