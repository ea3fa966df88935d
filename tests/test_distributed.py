"""CPU (gloo, world_size 2): the multi-rank path of bench.py — barrier-bracketed timing, max-over-ranks
elapsed time and summed bytes — with the oracle as the per-rank work (objects sharded, no data-path
collective).  Runs here without a GPU; the GPU bench uses the same Dist/timed_loop code and the same gloo group at
every N (the data path has no collective: DESIGN.md §6)."""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import time

    import numpy as np

    import bench
    from oracle.oracle import Oracle, OracleDecoder

    d = bench.Dist().init()
    orc = Oracle()
    k, L, n, m, B = 8, 512, 12, 8, 3
    rng = np.random.default_rng(100 + rank)  # each rank owns different objects
    src = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (B, n, k), dtype=np.uint8)
    results = []

    def step():
        out = []
        for o in range(B):
            coded = orc.encode(src[o], co[o])
            dec = OracleDecoder(L, k)
            for p in coded[:m]:
                dec.decode(p)
            out.append(dec.padded_payload())
        if rank == 1:
            time.sleep(0.02)  # the slow rank must set the reported time
        results.append(out)

    el = bench.timed_loop(step, steps=3, warmup=1, dist=d, sync=lambda: None)
    total = d.allreduce(float(bench.step_bytes(B, k, L, n) * 3), "sum")
    ok = all(np.array_equal(results[-1][o], src[o]) for o in range(B))
    q.put((rank, el, total, ok))
    d.close()


def test_two_rank_gloo_timing_and_aggregation():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, el0, tot0, ok0), (r1, el1, tot1, ok1) = res
    assert ok0 and ok1  # each rank decoded its own objects (full rank with 8 dense pieces of k=8)
    assert el0 == el1 and el0 >= 3 * 0.02  # max over ranks, the slow rank dominates
    import bench

    assert tot0 == tot1 == 2 * bench.step_bytes(3, 8, 512, 12) * 3


def test_step_bytes_matches_reference_counters():
    import bench

    k, L = 32, 1 << 20
    assert bench.encode_counter(k, L) == 34_603_040
    assert bench.decode_counter(k, L) == 33_555_456
    assert bench.step_bytes(16, k, L, 64) == 16 * (64 * 34_603_040 + 33_555_456)


def test_self_spawn_two_ranks_gloo():
    """`bench.py --gpus 2` with no launcher starts its own 2 ranks (fresh interpreters, RANK/WORLD_SIZE/MASTER_*
    set, rendezvous on 127.0.0.1) and rank 0 prints the one JSON line; here each rank's work is the C oracle
    over gloo (--workload oracle-cpu), the GPU bench takes the same path and the same group."""
    import json
    import subprocess
    import sys

    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2",
                        "--workload", "oracle-cpu", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["verified"]
    assert res["verified_per_rank"] == [True, True]
    assert res["world_size_initialised"] == 2  # torch.distributed.get_world_size() after init_process_group
    assert res["total_bytes"] == 2 * bench.step_bytes(3, 8, 512, 12) * 3
    assert abs(res["value"] - res["total_bytes"] / res["elapsed_s"] / bench.GIB) < 1e-3


def test_self_spawn_stops_ranks_when_one_fails():
    """A rank that dies before the rendezvous (test hook RLNC_BENCH_FAIL_RANK) makes the launcher stop the rank
    left waiting in init_process_group and return the dead rank's exit code instead of hanging."""
    import subprocess
    import sys

    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2",
                        "--workload", "oracle-cpu", "--steps", "2"], capture_output=True, text=True, timeout=120,
                       env=dict(env, RLNC_BENCH_FAIL_RANK="1"))
    assert r.returncode == 5


def test_config5_split_is_a_fixed_job():
    import bench

    a = bench.parse_args(["--workload", "config5"])
    assert (a.k, a.piece_bytes, a.coded, a.decode_from, a.objects, a.chunk) == (128, 1 << 16, 128, 128, 4096, 512)
    # objects per rank at N = 1..8 sum to the whole job
    for n in (1, 2, 3, 4, 8):
        per = [a.objects // n + (1 if r < a.objects % n else 0) for r in range(n)]
        assert sum(per) == 4096


def test_self_spawn_two_ranks_config5_split():
    """`--workload config5` is one fixed job split over the ranks (strong scaling): the same self-spawned harness
    with the oracle stand-in (`oracle-cpu-config5`), a job of 7 objects over 2 ranks (4 + 3)."""
    import json
    import subprocess
    import sys

    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2",
                        "--workload", "oracle-cpu-config5", "--objects", "7", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["scaling"] == "strong" and res["world_size_initialised"] == 2 and res["verified"]
    assert res["objects_total"] == 7 and res["objects_rank0"] == 4
    assert res["total_bytes"] == bench.step_bytes(7, 8, 512, 12) * 2


def test_single_rank_initialises_a_group():
    """N = 1 also reports the world size its process group initialised with (a free 127.0.0.1 port)."""
    import json
    import subprocess
    import sys

    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"),
                        "--workload", "oracle-cpu", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["world_size_initialised"] == 1


def _line(args):
    import json
    import subprocess
    import sys

    import bench

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py")] + args,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])


def test_same_process_group_backend_at_every_n():
    """A scaling curve compares like with like: the N = 1 and N = 2 lines report the same process-group backend
    (gloo: barrier and scalar results on the host, no RCCL streams beside the pipeline's), and the GPU run takes
    its group from the same Dist.init() as the oracle harness."""
    import inspect

    import bench

    one = _line(["--workload", "oracle-cpu", "--steps", "2", "--warmup", "1"])
    two = _line(["--gpus", "2", "--workload", "oracle-cpu", "--steps", "2", "--warmup", "1"])
    assert one["process_group_backend"] == two["process_group_backend"] == bench.HARNESS_BACKEND == "gloo"
    assert one["verified_per_rank"] == [True] and two["verified_per_rank"] == [True, True]
    src = inspect.getsource(bench.run_gpu)
    assert "dist.init()" in src and "nccl" not in src
