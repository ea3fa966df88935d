#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: device-resident RLNC encode+decode GiB/s, k=32 × 1 MiB, 1/2/4/8 MI355X.

Workloads (--workload):
  config2 (default; the metric's own shape, weak scaling): per GPU per step, --objects independent objects
    resident in HBM (default 32 × 32 MiB = 1 GiB of source, more than the 256 MiB Infinity Cache so source reads
    come from HBM; larger launches run faster per object, profiles/r01_launch_size.txt):
      * encode: 32 source pieces × 1 MiB → 64 full coded pieces (BASELINE configs[1]); one kernel launch for all
        objects (librlnc_hip rlnc_encode_batch);
      * decode: feed the first 32 coded pieces of every object to a fresh Decoder (configs[2]): exact
        diagonal-pivot elimination of the coefficient block per piece (device, gf_rref_batch_kernel), then
        T × data on the device, then the boundary-marker scan (rlnc_decode_batch_eliminate / _apply).
  config5 (BASELINE configs[4], strong scaling): ONE fixed job of 4,096 objects × k=128 × 64 KiB split over the
    N ranks; per object 128 coded pieces encoded and all 128 decoded; a step is the whole job (each rank's share
    in launches of ≤ 512 objects, pipelined like config2).
`value` = GiB/s in the reference's own byte counters (SURVEY.md §6 / BASELINE.md): per object
n × (k·L + k + L) for the n coded pieces (benches/full_rlnc_encoder.rs:111-113) + k·(k+L) for the decode
(benches/full_rlnc_decoder.rs:118), summed over all ranks, ÷ the max-over-ranks wall time of the timed steps.
Those counters charge the source k·L once per coded piece although one pass serves all n, so `value` is not
bytes moved: `breakdown.roundtrip_goodput_GiBps` (source bytes through encode + decode) sits beside it, and the
roofline is the kernel's own: GF(2^8) multiply-adds/s against the measured XOR3-issue ceiling (measure/).
Multi-GPU: objects are sharded across ranks, no data-path collective; the only collectives are the timing barrier
and the max/sum reductions of the result.  `--gpus N` without a launcher (WORLD_SIZE unset) starts N rank
processes itself (fresh interpreters, before any GPU call) with the same arguments.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RLNC encode+decode GiB/s, k=32 × 1 MiB, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)
MA_PER_XOR3 = 256  # GF(2^8) multiply-adds per v_bitop3 XOR3 of the bit-sliced kernel (measure/gf_ceiling.hip)
# the guide's VALU issue spec (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per
# SIMD at 2.4 GHz -> 1.2288 T XOR3/s x 256 multiply-adds = 314.6 T GF(2^8) multiply-adds/s
SPEC_XOR3_PER_S = 256 * 4 * 2.4e9 / 2
SPEC_PEAK_T_MA = SPEC_XOR3_PER_S * MA_PER_XOR3 / 1e12
HARNESS_BACKEND = "gloo"  # process-group backend at every N (Dist.init)
CPU_SHARE = 16  # host cores per GPU on the GPU box (os.cpu_count() there shows the whole machine)

WORKLOADS = {
    # name: k, L, coded n, decoded-from m, objects (per rank for config2, whole job for config5), chunk
    "config2": dict(k=32, L=1 << 20, n=64, m=32, objects=32, chunk=32, scaling="weak"),
    "config5": dict(k=128, L=1 << 16, n=128, m=128, objects=4096, chunk=512, scaling="strong"),
}


def encode_counter(k: int, L: int) -> int:
    """Bytes per coded piece, benches/full_rlnc_encoder.rs:111-113."""
    return k * L + k + L


def decode_counter(k: int, L: int) -> int:
    """Bytes per decoded object, benches/full_rlnc_decoder.rs:118."""
    return k * (k + L)


VARIANTS = ["perm", "nibble", "perm3", "wide2", "wide4", "bitsliced", "bitsliced-jump", "bitsliced-jump-shared",
            "bitsliced-jump-shared-8w", "bitsliced-jump-run"]
KERNELS = {"perm": "gf_matmul_perm_kernel", "nibble": "gf_matmul_nibble_kernel", "perm3": "gf_matmul_perm3_kernel",
           "wide2": "gf_matmul_wide_kernel", "wide4": "gf_matmul_wide_kernel",
           "bitsliced": "bs_index_kernel + gf_matmul_bs_kernel",
           "bitsliced-jump": "bsj_offset_kernel + gf_matmul_bsj_kernel",
           "bitsliced-jump-shared": "bsj_offset_kernel + gf_matmul_bsj_kernel<4, true>",
           "bitsliced-jump-shared-8w": "bsj_offset_kernel + gf_matmul_bsj_kernel<8, true>",
           "bitsliced-jump-run": "bsj_offset_kernel + gf_matmul_bsj_kernel<8, true, true>"}


def pmc_traffic(variant: str, B: int, k: int, L: int, n: int):
    """HBM bytes per encode launch (read + write) measured by rocprofv3 PMC passes (scripts/pmc_bench.sh ->
    scripts/pmc_traffic.py -> profiles/pmc_traffic.json, FETCH_SIZE x2 gfx950 correction applied), when the
    committed measurement is of this variant and shape; else None."""
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))[variant]
    except (OSError, KeyError, ValueError):
        return None, None
    if (rec["objects"], rec["k"], rec["piece_bytes"], rec["coded"]) != (B, k, L, n):
        return None, None
    return rec["hbm_read_bytes"] + rec["hbm_write_bytes"], rec["source"]


def step_bytes(objects: int, k: int, L: int, n: int) -> int:
    return objects * (n * encode_counter(k, L) + decode_counter(k, L))


# ------------------------------------------------------------------------------------------------------
# distributed timing harness (CPU-testable with gloo: tests/test_distributed.py)
# ------------------------------------------------------------------------------------------------------
class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        self.bar = None

    def init(self):
        """Initialise the process group -- at world size 1 too, on a free 127.0.0.1 port, so that every line reports
        the world size the group initialised with.  The backend is gloo at EVERY N: the data path has no collective
        (objects are sharded), so the group only carries the timing barrier and the scalar results, on
        the host.  Every rank synchronises its device right before the barrier, so a host barrier orders the ranks.
        An RCCL group would start RCCL's own streams on the 4 hardware queues the bench's three pipeline streams use
        (the pipelined step measured 4-5 % slower with an RCCL group at N = 1) and its barrier cost ~3.5 ms per call
        (profiles/r03_bench_pg_ab.txt); using it only at N > 1 would make the N = 1 point of a scaling curve cheaper
        than every other point."""
        import torch.distributed as dist

        if "MASTER_PORT" not in os.environ:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ["MASTER_PORT"] = str(_free_port())
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        backend = os.environ.get("RLNC_BENCH_PG", HARNESS_BACKEND)  # diagnostic override of the group's backend
        dist.init_process_group(backend=backend)
        self.pg = dist
        # with the diagnostic RCCL override the barrier still runs on a host group
        self.bar = dist.new_group(backend="gloo") if backend == "nccl" else None
        return self

    def backend(self):
        return self.pg.get_backend() if self.pg else None

    def initialised_world(self) -> int:
        return self.pg.get_world_size() if self.pg else 0

    def barrier(self):
        if self.pg:
            self.pg.barrier(group=self.bar)

    def allreduce(self, value: float, op: str) -> float:
        if not self.pg:
            return value
        import torch

        t = torch.tensor([value], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX if op == "max" else self.pg.ReduceOp.SUM, group=self.bar)
        return float(t.item())

    def allgather(self, value: float) -> list:
        """Every rank's value, in rank order (host group)."""
        if not self.pg:
            return [value]
        import torch

        out = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
        self.pg.all_gather(out, torch.tensor([value], dtype=torch.float64), group=self.bar)
        return [float(t.item()) for t in out]

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def timed_loop(step, steps: int, warmup: int, dist: Dist, sync) -> float:
    """W untimed steps, then exactly K steps bracketed by barrier + device sync; returns max-over-ranks s."""
    for _ in range(warmup):
        step()
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    return dist.allreduce(elapsed, "max")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` with no launcher: N fresh rank processes of this script (same arguments), one per GPU,
    rendezvous on 127.0.0.1.  This process never touches the GPU.  Returns the first nonzero exit code (the
    other ranks are stopped then, so a failed rank cannot leave the rest waiting in a barrier)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code and not rc:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ------------------------------------------------------------------------------------------------------
# CPU baseline: the oracle (C restatement of the reference's algorithm) — "port"
# ------------------------------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def _cpu_object_loop(k: int, L: int, n: int, m: int, seconds: float, seed: int):
    """One object's encode of n coded pieces (encoder.rs:128-144 per piece) + decode of m of them with a full-row
    RREF per piece (decoder.rs:96-118), repeated until `seconds`; returns (iterations, elapsed).  All the work is
    in the C oracle (ctypes releases the GIL, so threads run in parallel)."""
    import numpy as np

    from oracle.oracle import Oracle, OracleDecoder

    orc = Oracle()
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    coeffs = rng.integers(0, 256, (n, k), dtype=np.uint8)
    iters = 0
    t0 = time.perf_counter()
    while True:
        coded = orc.encode(src, coeffs)
        dec = OracleDecoder(L, k)
        for p in coded[:m]:
            dec.decode(p)
        dec.get_decoded_data()
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return iters, el


def cpu_baseline(k: int, L: int, n: int, m: int, seconds: float, threads: int = 1) -> dict:
    """Reference algorithm on the host: `threads` threads, one object each (the reference's default build is
    single-threaded per object; SURVEY.md §8d asks for one thread and for all cores, one object per thread); same
    byte counters as the GPU value."""
    import threading

    from oracle.oracle import Oracle

    res = [None] * threads

    def work(t):
        res[t] = _cpu_object_loop(k, L, n, m, seconds, 0x524C4E43 + t)

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    iters = sum(r[0] for r in res)
    value = iters * (n * encode_counter(k, L) + decode_counter(k, L)) / el / GIB
    how = "single thread" if threads == 1 else f"{threads} threads, one object each"
    return {
        "value": round(value, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{iters} x (1 object k={k} L={L}: encode {n} coded pieces + decode {m} with per-piece "
                  f"full-row RREF), {el:.1f} s, {how}, oracle/liboracle.so ({Oracle().simd_variant()}) "
                  f"on {cpu_model()}",
    }


# ------------------------------------------------------------------------------------------------------
# the GF(2^8) multiply-add ceiling, measured live (measure/gf_ceiling.hip)
# ------------------------------------------------------------------------------------------------------
def xor3_ceiling() -> dict | None:
    """Chip-wide v_bitop3 XOR3 issue rate (best of 2 and 4 waves per SIMD, random operands) × 256 multiply-adds
    per XOR3: the peak of the bit-sliced design.  None if the microbenchmark is not built."""
    path = os.path.join(ROOT, "measure", "libgf_ceiling.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.gf_xor3_issue_rate.restype = ctypes.c_double
    lib.gf_xor3_issue_rate.argtypes = [ctypes.c_int, ctypes.c_int]
    rates = {w: lib.gf_xor3_issue_rate(w, 200000) for w in (2, 4)}
    if min(rates.values()) <= 0:
        return None
    best = max(rates.values())
    return {"xor3_per_s": {str(w): round(r / 1e12, 4) for w, r in rates.items()},
            "xor3_unit": "T wave64 instructions/s (whole device)",
            "peak_T_ma_per_s": round(best * MA_PER_XOR3 / 1e12, 2),
            "how": "measure/gf_ceiling.hip: only independent v_bitop3_b32 XOR3s, 4 VGPR banks, random operands, "
                   "2 and 4 waves per SIMD on every CU, HIP events around a ~30 ms launch; × 256 GF(2^8) "
                   "multiply-adds per XOR3 (8 XOR3s add c·x into the 8 bit-planes of 64 lanes × 32 bytes)"}


def hbm_ceiling(objects: int, k: int, L: int) -> dict | None:
    """HBM rates of this box with no GF arithmetic (measure/hbm_ceiling.hip): a float4 copy, a contiguous read and
    the single-pass encoder's own access pattern (k rows of one 4 KiB column block per workgroup, XOR for the
    product).  None if the microbenchmark is not built."""
    path = os.path.join(ROOT, "measure", "libhbm_ceiling.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.hbm_rates.restype = ctypes.c_int
    lib.hbm_rates.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(ctypes.c_double)]
    r = (ctypes.c_double * 4)()
    if lib.hbm_rates(objects, k, L, r) != 0:
        return None
    return {"copy_GBps": round(r[0], 1), "read_GBps": round(r[1], 1), "pattern_read_GBps": round(r[2], 1),
            "pattern_compulsory_GBps": round(r[3], 1),
            "how": f"measure/hbm_ceiling.hip over {objects} x {k} x {L} B (> the 256 MiB Infinity Cache): 16-B/lane "
                   "copy (read+write bytes), contiguous read, and the single-pass encode's access pattern with XOR "
                   "in place of the GF product; median of 7 launches"}


# ------------------------------------------------------------------------------------------------------
# GPU run
# ------------------------------------------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 30 for config2, 5 for config5)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 5 for config2, 2 for config5)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS) + ["oracle-cpu", "oracle-cpu-config5"], default="config2",
                    help="config2: the metric's shape, objects per GPU (weak scaling); config5: BASELINE configs[4], "
                         "4,096 objects split over the ranks (strong scaling); oracle-cpu / oracle-cpu-config5: the "
                         "harness alone with the C oracle as each rank's work and gloo (tests), per-rank objects / "
                         "a fixed job split over the ranks")
    ap.add_argument("--objects", type=int, default=None,
                    help="config2: objects per GPU per step (32: profiles/r01_launch_size.txt); config5: the whole job")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--piece-bytes", type=int, default=None)
    ap.add_argument("--coded", type=int, default=None)
    ap.add_argument("--decode-from", type=int, default=None)
    ap.add_argument("--chunk", type=int, default=None, help="objects per launch (config5: 512)")
    ap.add_argument("--variant", type=int, default=8, help="matmul kernel variant: 8 as 7 with 64-row tiles of 8 waves above 32 output rows and a barrier every third row (default), 9 as 8 with column runs (a workgroup walks up to 8 column blocks, one prologue per run), 7 bit-sliced, one code block per coefficient, combinations shared through LDS, 6 the same without sharing, 5 bit-sliced relative XOR, 0 perm, 1 nibble-LDS, 2 perm3, 3/4 wide")
    ap.add_argument("--tile-rows", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the live XOR3-issue ceiling microbenchmark")
    ap.add_argument("--cpu-threads", type=int, default=CPU_SHARE,
                    help="threads of the CPU-share baseline (one object each; the GPU box grants 16 host cores per GPU)")
    ap.add_argument("--encode-only", action="store_true", help="diagnostic: time only the encode launch")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="1: the decoder's elimination (reads only the coded pieces' coefficient headers, written "
                         "first) runs on a second stream while the encode's data work runs; 2: as 1, and successive "
                         "launches overlap (two buffer sets: launch i+1's encode runs beside launch i's decode); 0: serial")
    ap.add_argument("--breakdown-steps", type=int, default=24,
                    help="--pipeline 2: launches of the pipeline-1 form run before the timed loop for the per-part times")
    ap.add_argument("--no-plan", action="store_true",
                    help="A/B: the encode launch and the decode's data side write their own code-block address streams "
                         "(the offset kernel in front of each product on its stream) instead of taking the ones written "
                         "ahead on the side stream")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay each step as one captured HIP graph (the kernels of a step, launched together; "
                         "the launch groups take the --pipeline 1 form: --pipeline 2 overlaps eager launches only)")
    args = ap.parse_args(argv)
    if args.workload in WORKLOADS:
        w = WORKLOADS[args.workload]
        for name, key in [("k", "k"), ("piece_bytes", "L"), ("coded", "n"), ("decode_from", "m"),
                          ("objects", "objects"), ("chunk", "chunk")]:
            if getattr(args, name) is None:
                setattr(args, name, w[key])
    big = args.workload == "config5"
    if args.steps is None:
        args.steps = 5 if big else 30
    if args.warmup is None:
        args.warmup = 2 if big else 5
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    dist = Dist()
    if os.environ.get("RLNC_BENCH_FAIL_RANK") == str(dist.rank):  # test hook: a rank dying before rendezvous
        sys.exit(5)
    assert dist.world == args.gpus or (dist.world == 1 and args.gpus == 1), \
        f"--gpus {args.gpus} but WORLD_SIZE={dist.world}"
    if args.workload.startswith("oracle-cpu"):
        return run_oracle_cpu(args, dist)
    return run_gpu(args, dist)


def run_oracle_cpu(args, dist: Dist):
    """The harness alone (spawn, rendezvous, barrier-bracketed steps, max-over-ranks time, summed bytes, one JSON
    line from rank 0) with the C oracle as each rank's work, over gloo: tests/test_distributed.py."""
    import numpy as np

    from oracle.oracle import Oracle, OracleDecoder

    dist.init()
    orc = Oracle()
    k, L, n, m, B = 8, 512, 12, 8, 3
    strong = args.workload == "oracle-cpu-config5"
    if strong:  # config5's split: a fixed job of J objects over the ranks (the first J % N ranks take one more)
        J = args.objects or 7
        B = J // dist.world + (1 if dist.rank < J % dist.world else 0)
    rng = np.random.default_rng(100 + dist.rank)  # each rank owns different objects
    src = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (B, n, k), dtype=np.uint8)
    last = []

    def step():
        out = []
        for o in range(B):
            coded = orc.encode(src[o], co[o])
            dec = OracleDecoder(L, k)
            for p in coded[:m]:
                dec.decode(p)
            out.append(dec.padded_payload())
        last[:] = out

    elapsed = timed_loop(step, args.steps, args.warmup, dist, lambda: None)
    total = dist.allreduce(float(step_bytes(B, k, L, n) * args.steps), "sum")
    total_objs = dist.allreduce(float(B), "sum")
    ok_rank = dist.allgather(float(all(np.array_equal(last[o], src[o]) for o in range(B))))
    ok = all(v == 1.0 for v in ok_rank)
    if dist.rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(total / elapsed / GIB, 6), "unit": "GiB/s",
                          "n_gpus": dist.world, "world_size_initialised": dist.initialised_world(),
                          "process_group_backend": dist.backend(), "verified_per_rank": [bool(v) for v in ok_rank],
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
                          "scaling": "strong" if strong else "weak", "elapsed_s": elapsed, "total_bytes": total,
                          "verified": bool(ok), "objects_total": int(total_objs), "objects_rank0": B,
                          "config": {"workload": "oracle-cpu harness test" + (" (fixed job split)" if strong else "")}}),
              flush=True)
    dist.close()
    if not ok:
        sys.exit(3)


def run_gpu(args, dist: Dist):
    import numpy as np
    import torch

    # the rank's device, chosen here in the fresh rank process (the spawning parent never touches the GPU): local
    # rank modulo the devices this process sees, so N ranks on a box with fewer GPUs share them (two ranks on the one
    # GPU of a test lease: tests/test_gpu_multirank.py); one rank per GPU on a full node
    device = dist.local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    dist.init()

    import rlnc_amd
    from rlnc_amd import batch

    wl = WORKLOADS[args.workload]
    k, L, n, m = args.k, args.piece_bytes, args.coded, args.decode_from
    if wl["scaling"] == "weak":
        objs = args.objects  # per rank
    else:  # a fixed job split over the ranks (the last ranks take one fewer when it does not divide)
        objs = args.objects // dist.world + (1 if dist.rank < args.objects % dist.world else 0)
    C = min(args.chunk, objs)  # objects per launch
    chunks = [(c0, min(objs, c0 + C)) for c0 in range(0, objs, C)]
    ctx = rlnc_amd.Context(device)
    ctx.set_kernel_variant(args.variant, args.tile_rows)
    dev = torch.device("cuda", device)

    # synthetic objects of the named shape, generated on device; coefficients from a host RNG (like
    # rng.fill_bytes in the reference) and uploaded before timing
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x524C4E43 + dist.rank)
    src = torch.randint(0, 256, (objs, k, L), dtype=torch.uint8, device=dev, generator=gen)
    coeffs = torch.from_numpy(np.random.default_rng(1000 + dist.rank).integers(0, 256, (objs, n, k),
                                                                                 dtype=np.uint8)).to(dev)

    def buffers(B):
        return dict(pieces=torch.empty((B, n, k + L), dtype=torch.uint8, device=dev),
                    # the encode's code-block address stream, written ahead on the side stream (encode_batch_prepare)
                    plan=torch.empty(batch.encode_plan_bytes(k, B, n), dtype=torch.uint8, device=dev),
                    # the decode's T x data address stream, written on the side stream behind the elimination
                    dplan=torch.empty(batch.decode_apply_plan_bytes(k, m, B), dtype=torch.uint8, device=dev),
                    decoded=torch.empty((B, k, L), dtype=torch.uint8, device=dev),
                    pst=torch.empty((B, m), dtype=torch.int32, device=dev),
                    ost=torch.empty(B, dtype=torch.int32, device=dev),
                    dl=torch.empty(B, dtype=torch.int64, device=dev),
                    T=torch.empty((B, k, m), dtype=torch.uint8, device=dev),
                    rank=torch.empty(B, dtype=torch.int32, device=dev),
                    obj=(0, 0))

    sets = [buffers(C)]
    enc_events, dec_events, apply_events, plan_events = [], [], [], []
    ctx_side = rlnc_amd.Context(device) if args.pipeline else None
    if ctx_side is not None:
        ctx_side.set_kernel_variant(args.variant, args.tile_rows)  # the plan is laid out for the launch's variant
    side = torch.cuda.Stream(dev) if args.pipeline else None
    ev_start, ev_elim, ev_plan = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()

    def views(S, c0, c1):
        b = c1 - c0
        return (src[c0:c1], coeffs[c0:c1], S["pieces"][:b], S["decoded"][:b], S["pst"][:b], S["ost"][:b],
                S["dl"][:b], S["T"][:b], S["rank"][:b])

    # one launch group = one chunk of objects: encode then decode, HIP events on the launch stream bracket each
    # part (pipelined: the encode part includes the concurrent elimination's interference, the decode part any
    # wait for it)
    def launch_serial(c0, c1, S, isolate=False):
        """isolate (the pipeline-1 breakdown groups behind the rooflines): the launch stream also waits for the
        elimination before the encode, so the encode and decode windows each hold their kernels alone -- no
        elimination sharing the CUs with the encode, no cross-stream wait inside the decode window."""
        s_, co, pieces, decoded, pst, ost, dl, T, rank = views(S, c0, c1)
        received = pieces[:, :m]
        e0, e1, ea, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        if args.pipeline:
            # side stream: the encode's code-block address stream, the coded pieces' headers (bytes 0..k of each
            # piece), then the elimination over them; launch stream: the data bytes k.. of the same pieces (disjoint
            # bytes), concurrently.  e0 is recorded once the address stream is ready, so the encode part is the
            # product kernel alone (the launches rocprofv3 attributes to gf_matmul_bsj_kernel)
            ev_start.record()
            with torch.cuda.stream(side):
                side.wait_event(ev_start)
                if not args.no_plan:
                    # the address stream's own launch, timed on the side stream it runs on (outside e0..e1)
                    p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    p0.record()
                    batch.encode_batch_prepare(s_, co, pieces, S["plan"], ctx_side)
                    p1.record()
                    plan_events.append((p0, p1))
                ev_plan.record()
                batch.encode_batch_headers(co, pieces, ctx_side)
                if not args.encode_only:
                    batch.decode_batch_eliminate(received, k, T, pst, rank, ctx_side)
                    if not args.no_plan:
                        batch.decode_batch_apply_prepare(received, k, T, decoded, S["dplan"], ctx_side)
                ev_elim.record()
            torch.cuda.current_stream().wait_event(ev_plan)
            if isolate:
                torch.cuda.current_stream().wait_event(ev_elim)
            e0.record()
            if args.no_plan:
                batch.encode_batch_data(s_, co, pieces, ctx)
            else:
                batch.encode_batch_data_planned(s_, co, pieces, S["plan"], ctx)
            if args.encode_only:
                torch.cuda.current_stream().wait_event(ev_elim)
        else:
            e0.record()
            batch.encode_batch(s_, co, pieces, ctx)
        e1.record()
        if not args.encode_only:
            if args.pipeline:
                if not isolate:
                    torch.cuda.current_stream().wait_event(ev_elim)
                ea.record()  # the decode's data side alone: T x data and the marker scan (+ the address launch: --no-plan)
                if args.no_plan:
                    batch.decode_batch_apply(received, k, T, rank, decoded, ost, dl, ctx)
                else:
                    batch.decode_batch_apply_planned(received, k, T, rank, decoded, ost, dl, S["dplan"], ctx)
                apply_events.append((ea, e2))
            else:
                batch.decode_batch_device(received, k, decoded, pst, ost, dl, ctx)
        e2.record()
        S["obj"] = (c0, c1)
        enc_events.append((e0, e1))
        dec_events.append((e1, e2))

    def step_serial():
        for c0, c1 in chunks:
            launch_serial(c0, c1, sets[0])

    # --pipeline 2: launch group i uses buffer set i % 2; its headers + elimination (side stream), encode data
    # (launch stream) and decode data side (decode stream) wait only for group i-2's decode to release that
    # set, so group i+1's encode fills the GPU beside group i's decode (no tail or launch gaps between the big
    # kernels).  Every group still does all of its work.
    pipelined = args.pipeline == 2 and not args.encode_only and not args.graph  # a graph replays the serial step
    if pipelined:
        sets.append(buffers(C))
        ctx_dec = rlnc_amd.Context(device)
        ctx_dec.set_kernel_variant(args.variant, args.tile_rows)
        s_dec = torch.cuda.Stream(dev)
        ev_done = [torch.cuda.Event(), torch.cuda.Event()]
        ev_enc = [torch.cuda.Event(), torch.cuda.Event()]
        ev_el = [torch.cuda.Event(), torch.cuda.Event()]
        ev_pl = [torch.cuda.Event(), torch.cuda.Event()]
        count = [0]

        def launch_pipelined(c0, c1):
            i = count[0]
            count[0] += 1
            bi = i % 2
            S = sets[bi]
            s_, co, pieces, decoded, pst, ost, dl, T, rank = views(S, c0, c1)
            rec = pieces[:, :m]
            with torch.cuda.stream(side):
                # the address stream of set bi is free once group i-2's encode has run: written here, behind group
                # i-1's elimination on the side stream, long before the launch stream reaches group i's encode
                if i >= 2:
                    side.wait_event(ev_enc[bi])
                if not args.no_plan:
                    batch.encode_batch_prepare(s_, co, pieces, S["plan"], ctx_side)
                ev_pl[bi].record()
                if i >= 2:
                    side.wait_event(ev_done[bi])
                batch.encode_batch_headers(co, pieces, ctx_side)
                batch.decode_batch_eliminate(rec, k, T, pst, rank, ctx_side)
                if not args.no_plan:
                    batch.decode_batch_apply_prepare(rec, k, T, decoded, S["dplan"], ctx_side)
                ev_el[bi].record()
            if i >= 2:
                torch.cuda.current_stream().wait_event(ev_done[bi])
            torch.cuda.current_stream().wait_event(ev_pl[bi])
            if args.no_plan:
                batch.encode_batch_data(s_, co, pieces, ctx)
            else:
                batch.encode_batch_data_planned(s_, co, pieces, S["plan"], ctx)
            ev_enc[bi].record()
            with torch.cuda.stream(s_dec):
                s_dec.wait_event(ev_enc[bi])
                s_dec.wait_event(ev_el[bi])
                if args.no_plan:
                    batch.decode_batch_apply(rec, k, T, rank, decoded, ost, dl, ctx_dec)
                else:
                    batch.decode_batch_apply_planned(rec, k, T, rank, decoded, ost, dl, S["dplan"], ctx_dec)
                ev_done[bi].record()
            S["obj"] = (c0, c1)

        def step_pipelined():
            for c0, c1 in chunks:
                launch_pipelined(c0, c1)

    run = step_pipelined if pipelined else step_serial
    skip = args.warmup * len(chunks)
    if args.graph:
        # eager warmup steps (they also give the per-kernel breakdown), then capture one step's launches into
        # a graph: the timed steps replay it, identical kernels and work, without per-launch host overhead
        eager = max(args.warmup, 2)
        for _ in range(eager):
            step_serial()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step_serial()
        run = g.replay
        for evs in (enc_events, dec_events, apply_events, plan_events):
            del evs[eager * len(chunks):]  # events recorded under capture are graph nodes, not timestamps
        skip = len(chunks)  # the per-part times: the eager steps after the first
    elif pipelined:
        # the per-part times (encode launch for the roofline, decode) come from pipeline-1 launch groups run
        # before the timed loop (the first 6 discarded: clocks and caches settle): a kernel's own duration, not
        # its overlap with the next group's kernels
        for i in range(args.breakdown_steps + 6):
            c0, c1 = chunks[i % len(chunks)]
            launch_serial(c0, c1, sets[0], isolate=True)
        torch.cuda.synchronize()
        skip = 6
    elapsed = timed_loop(run, args.steps, args.warmup, dist, torch.cuda.synchronize)
    torch.cuda.synchronize()

    def verified(S):
        # every full-rank object of the last launch group that used this set decodes to its source
        c0, c1 = S["obj"]
        b = c1 - c0
        pst, ost = S["pst"][:b].cpu().numpy(), S["ost"][:b].cpu().numpy()
        good = True
        for o in range(b):
            if (pst[o] == 0).sum() == k:
                good = good and torch.equal(S["decoded"][o], src[c0 + o])
            else:
                good = good and int(ost[o]) == 10  # NotAllPiecesReceivedYet (rank-deficient draw)
        return good and bool((pst == 0).sum(axis=1).max() == k)

    ok = True
    if not args.encode_only:
        for S in sets:
            ok = ok and verified(S)
    timed_enc = enc_events[skip:] or enc_events
    enc_ms = sum(a.elapsed_time(b) for a, b in timed_enc) / len(timed_enc)
    timed_dec = dec_events[skip:] or dec_events
    dec_ms = sum(a.elapsed_time(b) for a, b in timed_dec) / len(timed_dec)

    def mean_ms(evs):
        evs = evs[skip:] or evs
        return sum(a.elapsed_time(b) for a, b in evs) / len(evs) if evs else None

    apply_ms = mean_ms(apply_events)  # pipeline-1 groups only (launch_serial with --pipeline >= 1)
    plan_ms = mean_ms(plan_events)
    ok_rank = dist.allgather(float(ok))
    ok = all(v == 1.0 for v in ok_rank)
    enc_ms_rank = dist.allgather(enc_ms)
    dec_ms_rank = dist.allgather(dec_ms)

    per_rank_bytes = step_bytes(objs, k, L, n) if not args.encode_only else objs * n * encode_counter(k, L)
    total_bytes = dist.allreduce(float(per_rank_bytes * args.steps), "sum")
    total_objs = dist.allreduce(float(objs), "sum")
    value = total_bytes / elapsed / GIB

    # roofline of the dominant kernel (the encode matmul, one launch per launch group) from HIP events.  The
    # kernel is bound by VALU issue, not HBM: `achieved` = its GF(2^8) multiply-adds per second,
    # `peak` = the live XOR3-issue ceiling of the bit-sliced design; the HBM view (compulsory bytes: source once
    # + coded pieces written, and the PMC-measured traffic) sits beside it.
    B = C
    ma_per_launch = B * n * k * L                    # GF(2^8) multiply-adds per encode launch
    achieved = ma_per_launch / (enc_ms * 1e-3) / 1e12
    enc_alg = B * n * encode_counter(k, L)           # reference-counter bytes per launch
    enc_compulsory = B * (k * L + n * (k + L))       # source read once + coded pieces written
    variant = VARIANTS[args.variant]
    traffic, traffic_src = pmc_traffic(variant, B, k, L, n)
    # the product kernel alone is inside e0..e1 unless --no-plan puts the address launch in front of it
    enc_kernel = KERNELS[variant] if args.no_plan else KERNELS[variant].replace("bsj_offset_kernel + ", "")
    ceiling = None if args.no_ceiling else xor3_ceiling()
    live = ceiling["peak_T_ma_per_s"] if ceiling else None
    roofline = {
        "bound": "valu",
        "achieved": round(achieved, 2),
        # peak = the guide's VALU issue rate (MI355X_MICROARCH.md: one wave64 instruction per 2 cycles per SIMD at
        # 2.4 GHz, 1,024 SIMDs) x 256 GF(2^8) multiply-adds per XOR3
        "peak": round(SPEC_PEAK_T_MA, 2),
        "unit": "T GF(2^8) multiply-adds/s",
        "frac": round(achieved / SPEC_PEAK_T_MA, 4),
        "frac_definition": "achieved / peak, peak = the guide's VALU issue rate (since round 5; rounds 1-4 reported "
                           "frac against the live XOR3 ceiling, which is frac_live now)",
        # beside it, the live XOR3-issue ceiling measured in this run (measure/gf_ceiling.hip: independent XOR3s only,
        # 0.75-0.77 of the spec rate -- the clock under load and three-source issue)
        "peak_live": live,
        "frac_live": round(achieved / live, 4) if live else None,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel": f"{enc_kernel} (encode: {n} coded pieces x {B} objects per launch)",
        "kernel_ms": round(enc_ms, 4),
        # the code-block address launch (rlnc_encode_batch_prepare) on the side stream, outside kernel_ms
        "address_stream_ms": round(plan_ms, 4) if plan_ms is not None else None,
        "kernel_ms_how": (("HIP events around the encode launch on its stream, in pipeline-1 launch groups run "
                          "before the timed loop, the elimination finished before it (the kernel alone)")
                         if pipelined else
                         ("HIP events around the encode launch on its stream (the elimination beside it)")
                         if args.pipeline else "HIP events around the encode launch")
                        + (" (--graph 1: in the eager steps before the capture)" if args.graph else ""),
        "multiply_adds_per_launch": ma_per_launch,
        "ceiling": ceiling,
        "hbm": {"compulsory_bytes": enc_compulsory,
                "compulsory_GBps": round(enc_compulsory / (enc_ms * 1e-3) / 1e9, 1),
                "peak_GBps": HBM_PEAK_GBS,
                "compulsory_frac": round(enc_compulsory / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic_over_compulsory": round(traffic / enc_compulsory, 4) if traffic else None},
        "refcounter": {"bytes_per_launch": enc_alg, "GBps": round(enc_alg / (enc_ms * 1e-3) / 1e9, 1),
                       "note": "the reference's encoder byte counter charges the source once per coded piece; "
                               f"{n} coded pieces share one source pass, so this is not a bandwidth"},
    }

    # the decode's data side (its own roofline): decoded rows = T (k x m) x the m received pieces' data,
    # k * m * L multiply-adds per object in the same bit-sliced engine (32-row tiles: the 4-wave shared program), timed
    # with HIP events on its stream around rlnc_decode_batch_apply in the pipeline-1 groups (after the wait for the
    # elimination, so only the apply's launches: its address launch, the product and the marker scan)
    roofline_decode = None
    if apply_ms:
        ma_dec = B * k * m * L
        dec_achieved = ma_dec / (apply_ms * 1e-3) / 1e12
        dec_compulsory = B * (m * L + k * L)  # received data read once + decoded rows written
        dtraffic, dtraffic_src = pmc_traffic("decode:" + variant, B, k, L, n)
        roofline_decode = {
            "bound": "valu",
            "achieved": round(dec_achieved, 2),
            "peak": round(SPEC_PEAK_T_MA, 2),
            "unit": "T GF(2^8) multiply-adds/s",
            "frac": round(dec_achieved / SPEC_PEAK_T_MA, 4),
            "frac_live": round(dec_achieved / live, 4) if live else None,
            "traffic": dtraffic,
            "traffic_source": dtraffic_src,
            "kernel": (("bsj_offset_kernel + " if args.no_plan else "") +
                       f"gf_matmul_bsj_kernel<4, true> + final_len_scan_kernel (decode data side: "
                       f"{k} decoded rows from {m} received pieces x {B} objects per launch"
                       + ("" if args.no_plan else "; its address stream written ahead on the side stream") + ")"),
            "kernel_ms": round(apply_ms, 4),
            "kernel_ms_how": "HIP events on the launch stream around rlnc_decode_batch_apply, in pipeline-1 launch "
                             "groups run before the timed loop (the elimination finished before the group's encode)"
                             if pipelined else "HIP events around rlnc_decode_batch_apply after its wait for the "
                             "elimination",
            "multiply_adds_per_launch": ma_dec,
            "hbm": {"compulsory_bytes": dec_compulsory,
                    "compulsory_GBps": round(dec_compulsory / (apply_ms * 1e-3) / 1e9, 1),
                    "compulsory_frac": round(dec_compulsory / (apply_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "traffic_over_compulsory": round(dtraffic / dec_compulsory, 4) if dtraffic else None},
        }

    # supplementary HBM roofline: the same source, ONE coded piece per object per launch (configs[1]'s encode
    # at one output row, ~1 multiply-add per source byte: the HBM-bound form of the north star's "encode at
    # k=32 x 1 MiB"); not part of `value`
    single = None
    if not args.encode_only and args.workload == "config2":
        c0, c1 = chunks[0]
        co1 = coeffs[c0:c1, :1].contiguous()
        out1 = torch.empty((c1 - c0, 1, k + L), dtype=torch.uint8, device=dev)
        # REPS back-to-back launches between one pair of events, so the ~10 us of launch latency of a lone ~190 us
        # launch is not charged to HBM (rocprofv3's per-launch duration is the cross-check)
        reps = 10
        for _ in range(2):
            batch.encode_batch(src[c0:c1], co1, out1, ctx)
        ts = []
        for r in range(3):
            a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                batch.encode_batch(src[c0:c1], co1, out1, ctx)
            b_.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b_) / reps)
        ms1 = sorted(ts)[len(ts) // 2]
        S0 = sets[0]  # holds the timed encode of chunk 0 (config2 has one launch group per step)
        ok1 = S0["obj"] == (c0, c1) and torch.equal(out1[:, 0, k:], S0["pieces"][: c1 - c0, 0, k:])
        read1 = (c1 - c0) * (k * L + k)
        single = {"coded_per_pass": 1, "kernel": "gf_matmul_stream3_kernel<1, 1, 2, true>", "ms": round(ms1, 4),
                  "ms_how": f"HIP events around {reps} back-to-back launches, median of 3",
                  "source_read_GBps": round(read1 / ms1 / 1e6, 1),
                  "read_frac": round(read1 / ms1 / 1e6 / HBM_PEAK_GBS, 4),
                  "compulsory_GBps": round((read1 + (c1 - c0) * (k + L)) / ms1 / 1e6, 1), "verified": bool(ok1)}
        hc = None if args.no_ceiling else hbm_ceiling(c1 - c0, k, L)
        if hc:
            single["ceiling"] = hc
            single["frac_of_pattern_ceiling"] = round(read1 / ms1 / 1e6 / hc["pattern_read_GBps"], 4)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": dist.world,
        "world_size_initialised": dist.initialised_world(),
        "process_group_backend": dist.backend(),
        "verified_per_rank": [bool(v) for v in ok_rank],
        "kernel_ms_per_rank": [round(v, 4) for v in enc_ms_rank],
        "decode_ms_per_rank": [round(v, 4) for v in dec_ms_rank],
        # 1: the device runs 16-byte vector memory instructions at any byte address (probed at context creation;
        # misaligned rows take the vector kernels directly), 0: they go through realigning copies
        "unaligned_vector_access": int(ctx.lib.rlnc_device_unaligned_vector_access(device)),
        "device_per_rank": [int(v) for v in dist.allgather(float(device))],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: uniform random source bytes (torch generator, seeded per rank), coefficients "
                "uniform bytes from a seeded host RNG",
        "config": {
            "workload": (f"configs[1]+[2]: per object encode k={k} x {L} B -> {n} coded pieces + decode from the "
                         f"first {m}; {objs} objects per GPU per step") if args.workload == "config2" else
                        (f"configs[4]: {int(total_objs)} objects x k={k} x {L} B split over {dist.world} rank(s) "
                         f"({objs} on rank {dist.rank}), encode {n} coded + decode {m} per object, "
                         f"launches of {C} objects; one step = the whole job"),
            "k": k, "piece_bytes": L, "coded_per_object": n, "decoded_from": m, "objects_per_gpu": objs,
            "objects_total": int(total_objs), "objects_per_launch": C,
            "parallelism": f"objects sharded over {dist.world} rank(s), no data-path collective",
            "kernel_variant": variant,
            "encode_address_stream": "launch stream (--no-plan)" if args.no_plan else
                                     "written ahead on the side stream (rlnc_encode_batch_prepare)",
            "pipeline": {0: "serial", 1: "elimination on a side stream concurrent with the encode data work",
                         2: "elimination beside the encode data work, and launch group i+1's encode beside group "
                            "i's decode (two buffer sets)"}[1 if args.pipeline == 2 and not pipelined else args.pipeline]
                        + (", replayed as one captured HIP graph per step" if args.graph else ""),
        },
        "roofline": roofline,
        "roofline_decode": roofline_decode,
        "hbm_single_pass_encode": single,
        "cpu_baseline": None,
        "breakdown": {
            "encode_kernel_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "decode_apply_ms": round(apply_ms, 4) if apply_ms is not None else None,
            "encode_T_ma_per_s": round(achieved, 2),
            "encode_GiBps_refcounter": round(B * n * encode_counter(k, L) / (enc_ms * 1e-3) / GIB, 1),
            "decode_GiBps_refcounter": round(B * decode_counter(k, L) / (dec_ms * 1e-3) / GIB, 2) if dec_ms else None,
            "roundtrip_goodput_GiBps": round(total_objs * k * L * args.steps / elapsed / GIB, 2),
            "roundtrip_goodput_note": "source bytes encoded and decoded per second, all ranks (not reference counters)",
            "verified": ok,
        },
    }
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(k, L, n, m, args.cpu_seconds)
        result["vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
        if args.cpu_threads > 1:
            # the same on the host cores one GPU gets on the box (16; os.cpu_count() there is the whole machine's,
            # which this process may not use), one object per thread
            threads = min(args.cpu_threads, os.cpu_count() or 1)
            share = cpu_baseline(k, L, n, m, args.cpu_seconds, threads)
            share["host_cpus_visible"] = os.cpu_count()
            share["note"] = (f"{threads} threads = the GPU box's host-core share per GPU; the machine shows "
                             f"{os.cpu_count()} CPUs, shared by its 8 GPUs' jobs")
            result["cpu_baseline_cpu_share"] = share
            result["vs_cpu_baseline_cpu_share"] = round(value / share["value"], 1)
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()
    if not ok:
        print("VERIFICATION FAILED: decoded data does not match the source", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
