#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: device-resident RLNC encode+decode GiB/s, k=32 × 1 MiB, 1/2/4/8 MI355X.

One step = for each of --objects independent objects resident in HBM (default 32 × 32 MiB = 1 GiB of source per
GPU, more than the 256 MiB Infinity Cache so source reads come from HBM; larger launches run faster per object,
profiles/r01_launch_size.txt):
  * encode: 32 source pieces × 1 MiB → 64 full coded pieces (BASELINE configs[1]); one kernel launch for all
    objects (librlnc_hip rlnc_encode_batch);
  * decode: feed the first 32 coded pieces of every object to a fresh Decoder (configs[2]): exact
    diagonal-pivot elimination of the coefficient block per piece (device, gf_rref_batch_kernel), then
    T × data on the device, then the boundary-marker scan (rlnc_decode_batch_eliminate / _apply).
`value` = GiB/s in the reference's own byte counters (SURVEY.md §6 / BASELINE.md): per object
64 × (k·L + k + L) for the 64 coded pieces (benches/full_rlnc_encoder.rs:111-113) + k·(k+L) for the decode
(benches/full_rlnc_decoder.rs:118), summed over all ranks, ÷ the max-over-ranks wall time of the timed steps.
Multi-GPU: objects are sharded across ranks (weak scaling), no data-path collective; the only collectives
are the timing barrier and the max/sum reductions of the result.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RLNC encode+decode GiB/s, k=32 × 1 MiB, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)


def encode_counter(k: int, L: int) -> int:
    """Bytes per coded piece, benches/full_rlnc_encoder.rs:111-113."""
    return k * L + k + L


def decode_counter(k: int, L: int) -> int:
    """Bytes per decoded object, benches/full_rlnc_decoder.rs:118."""
    return k * (k + L)


VARIANTS = ["perm", "nibble", "perm3", "wide2", "wide4", "bitsliced", "bitsliced-jump", "bitsliced-jump-shared",
            "bitsliced-jump-shared-8w"]
KERNELS = {"perm": "gf_matmul_perm_kernel", "nibble": "gf_matmul_nibble_kernel", "perm3": "gf_matmul_perm3_kernel",
           "wide2": "gf_matmul_wide_kernel", "wide4": "gf_matmul_wide_kernel",
           "bitsliced": "bs_index_kernel + gf_matmul_bs_kernel",
           "bitsliced-jump": "bsj_offset_kernel + gf_matmul_bsj_kernel",
           "bitsliced-jump-shared": "bsj_offset_kernel + gf_matmul_bsj_kernel<4, true>",
           "bitsliced-jump-shared-8w": "bsj_offset_kernel + gf_matmul_bsj_kernel<8, true>"}


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

    def init(self, backend: str):
        if self.world > 1:
            import torch.distributed as dist

            dist.init_process_group(backend=backend)
            self.pg = dist
        return self

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def allreduce(self, value: float, op: str) -> float:
        if not self.pg:
            return value
        import torch

        dev = "cuda" if self.pg.get_backend() == "nccl" else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX if op == "max" else self.pg.ReduceOp.SUM)
        return float(t.item())

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
# GPU run
# ------------------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--objects", type=int, default=32, help="objects per GPU per step (32: profiles/r01_launch_size.txt)")
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--piece-bytes", type=int, default=1 << 20)
    ap.add_argument("--coded", type=int, default=64)
    ap.add_argument("--decode-from", type=int, default=32)
    ap.add_argument("--variant", type=int, default=8, help="matmul kernel variant: 8 as 7 with 64-row tiles of 8 waves above 32 output rows and a barrier every third row (default), 7 bit-sliced, one code block per coefficient, combinations shared through LDS, 6 the same without sharing, 5 bit-sliced relative XOR, 0 perm, 1 nibble-LDS, 2 perm3, 3/4 wide")
    ap.add_argument("--tile-rows", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the all-cores CPU baseline (one object each; the box's share is 16 cores per GPU)")
    ap.add_argument("--encode-only", action="store_true", help="diagnostic: time only the encode launch")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="1: the decoder's elimination (reads only the coded pieces' coefficient headers, written "
                         "first) runs on a second stream while the encode's data work runs; 2: as 1, and successive "
                         "steps overlap (two buffer sets: step i+1's encode runs beside step i's decode); 0: serial")
    ap.add_argument("--breakdown-steps", type=int, default=24,
                    help="--pipeline 2: steps of the pipeline-1 form run before the timed loop for the per-part times")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay each step as one captured HIP graph (the kernels of a step, launched together)")
    args = ap.parse_args()

    import numpy as np
    import torch

    dist = Dist()
    assert dist.world == args.gpus or (dist.world == 1 and args.gpus == 1), \
        f"--gpus {args.gpus} but WORLD_SIZE={dist.world} (launch with torch.distributed.run for N>1)"
    torch.cuda.set_device(dist.local_rank)
    dist.init("nccl")

    import rlnc_amd
    from rlnc_amd import batch

    k, L, n, m, B = args.k, args.piece_bytes, args.coded, args.decode_from, args.objects
    ctx = rlnc_amd.Context(dist.local_rank)
    ctx.set_kernel_variant(args.variant, args.tile_rows)
    dev = torch.device("cuda", dist.local_rank)

    # synthetic objects of the named shape, generated on device; coefficients from a host RNG (like
    # rng.fill_bytes in the reference) and uploaded before timing
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x524C4E43 + dist.rank)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=gen)
    coeffs = torch.from_numpy(np.random.default_rng(1000 + dist.rank).integers(0, 256, (B, n, k), dtype=np.uint8)).to(dev)
    pieces = torch.empty((B, n, k + L), dtype=torch.uint8, device=dev)
    decoded = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
    received = pieces[:, :m]
    piece_status = torch.empty((B, m), dtype=torch.int32, device=dev)
    object_status = torch.empty(B, dtype=torch.int32, device=dev)
    data_len = torch.empty(B, dtype=torch.int64, device=dev)

    enc_events = []
    dec_events = []
    # pipelined step: the coded pieces' headers are written first (one strided copy), then the decoder's
    # elimination — which reads nothing else — runs on a side stream (its own context) concurrently with the
    # encode's data work; the data side of the decode waits for both.  Same kernels, same bytes as serial.
    ctx_side = rlnc_amd.Context(dist.local_rank) if args.pipeline else None
    side = torch.cuda.Stream(dev) if args.pipeline else None
    ev_start, ev_elim = torch.cuda.Event(), torch.cuda.Event()
    T = torch.empty((B, k, m), dtype=torch.uint8, device=dev)
    rank = torch.empty(B, dtype=torch.int32, device=dev)

    def encode_launches():
        if args.pipeline:
            # side stream: the coded pieces' headers (bytes 0..k of each piece), then the elimination over them;
            # launch stream: the data bytes k.. of the same pieces (disjoint bytes), concurrently
            ev_start.record()
            with torch.cuda.stream(side):
                side.wait_event(ev_start)
                batch.encode_batch_headers(coeffs, pieces, ctx_side)
                if not args.encode_only:
                    batch.decode_batch_eliminate(received, k, T, piece_status, rank, ctx_side)
                ev_elim.record()
            batch.encode_batch_data(src, coeffs, pieces, ctx)
            if args.encode_only:
                torch.cuda.current_stream().wait_event(ev_elim)
        else:
            batch.encode_batch(src, coeffs, pieces, ctx)

    def decode_launches():
        if args.encode_only:
            return
        if args.pipeline:
            torch.cuda.current_stream().wait_event(ev_elim)
            batch.decode_batch_apply(received, k, T, rank, decoded, object_status, data_len, ctx)
        else:
            batch.decode_batch_device(received, k, decoded, piece_status, object_status, data_len, ctx)

    def step():
        # encode, then the device-side decode (elimination + T×data + marker scan), asynchronous; HIP events
        # on the launch stream bracket each part (pipelined: the encode part includes the concurrent elimination's
        # interference, the decode part any wait for it)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        encode_launches()
        e1.record()
        decode_launches()
        e2.record()
        enc_events.append((e0, e1))
        dec_events.append((e1, e2))

    # --pipeline 2: step i uses buffer set i % 2; its headers + elimination (side stream), encode data (launch
    # stream) and decode data side (decode stream) wait only for step i-2's decode to release that set, so step
    # i+1's encode fills the GPU beside step i's decode (no tail or launch gaps between the big kernels)
    if args.pipeline == 2 and not args.encode_only:
        sets = [dict(pieces=pieces, decoded=decoded, pst=piece_status, ost=object_status, dl=data_len, T=T, rank=rank)]
        sets.append(dict(pieces=torch.empty_like(pieces), decoded=torch.empty_like(decoded),
                         pst=torch.empty_like(piece_status), ost=torch.empty_like(object_status),
                         dl=torch.empty_like(data_len), T=torch.empty_like(T), rank=torch.empty_like(rank)))
        ctx_dec = rlnc_amd.Context(dist.local_rank)
        ctx_dec.set_kernel_variant(args.variant, args.tile_rows)
        s_dec = torch.cuda.Stream(dev)
        ev_done = [torch.cuda.Event(), torch.cuda.Event()]
        ev_enc = [torch.cuda.Event(), torch.cuda.Event()]
        ev_el = [torch.cuda.Event(), torch.cuda.Event()]
        count = [0]

        def step2():
            i = count[0]
            count[0] += 1
            bi = i % 2
            S = sets[bi]
            rec = S["pieces"][:, :m]
            with torch.cuda.stream(side):
                if i >= 2:
                    side.wait_event(ev_done[bi])
                batch.encode_batch_headers(coeffs, S["pieces"], ctx_side)
                batch.decode_batch_eliminate(rec, k, S["T"], S["pst"], S["rank"], ctx_side)
                ev_el[bi].record()
            if i >= 2:
                torch.cuda.current_stream().wait_event(ev_done[bi])
            batch.encode_batch_data(src, coeffs, S["pieces"], ctx)
            ev_enc[bi].record()
            with torch.cuda.stream(s_dec):
                s_dec.wait_event(ev_enc[bi])
                s_dec.wait_event(ev_el[bi])
                batch.decode_batch_apply(rec, k, S["T"], S["rank"], S["decoded"], S["ost"], S["dl"], ctx_dec)
                ev_done[bi].record()

    run = step2 if args.pipeline == 2 and not args.encode_only else step
    if args.graph:
        # eager warmup steps (they also give the per-kernel breakdown), then capture one step's launches into
        # a graph: the timed steps replay it, identical kernels and work, without per-launch host overhead
        for _ in range(max(args.warmup, 2)):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            encode_launches()
            decode_launches()
        run = g.replay
    if run is not step and not args.graph:
        # --pipeline 2: the per-part times (encode launch for the roofline, decode) come from pipeline-1 steps run
        # before the timed loop (the first 6 discarded: clocks and caches settle): a kernel's own duration, not its
        # overlap with the next step's kernels
        for _ in range(args.breakdown_steps + 6):
            step()
        torch.cuda.synchronize()
    elapsed = timed_loop(run, args.steps, args.warmup, dist, torch.cuda.synchronize)
    torch.cuda.synchronize()
    skip = 0 if args.graph else args.warmup  # graph mode: the eager warmup steps carry the breakdown
    def verified(vdec, vpst, vost):
        # every full-rank object decodes to its source
        pst, ost = vpst.cpu().numpy(), vost.cpu().numpy()
        good = True
        for o in range(B):
            if (pst[o] == 0).sum() == k:
                good = good and torch.equal(vdec[o], src[o])
            else:
                good = good and int(ost[o]) == 10  # NotAllPiecesReceivedYet (rank-deficient draw)
        return good and bool((pst == 0).sum(axis=1).max() == k)

    # correctness of what was timed: the last step's outputs (--pipeline 2: the last two steps', one per buffer set)
    ok = True
    if run is not step and not args.graph:  # --pipeline 2
        for S in sets:
            ok = ok and verified(S["decoded"], S["pst"], S["ost"])
        skip = 6
    elif not args.encode_only:
        ok = verified(decoded, piece_status, object_status)
    timed_enc = enc_events[skip:]
    enc_ms = sum(a.elapsed_time(b) for a, b in timed_enc) / len(timed_enc)
    timed_dec = dec_events[skip:]
    dec_ms = sum(a.elapsed_time(b) for a, b in timed_dec) / len(timed_dec)

    per_rank_bytes = step_bytes(B, k, L, n) if not args.encode_only else B * n * encode_counter(k, L)
    total_bytes = dist.allreduce(float(per_rank_bytes * args.steps), "sum")
    value = total_bytes / elapsed / GIB

    # roofline of the dominant kernel (the encode matmul, one launch per step) from HIP events
    enc_alg = B * n * encode_counter(k, L)           # reference counter bytes per launch
    enc_compulsory = B * (k * L + n * (k + L))       # source read once + coded pieces written
    achieved = enc_alg / (enc_ms * 1e-3) / 1e9
    ma_per_launch = B * n * k * L                    # GF(2^8) multiply-adds per launch
    variant = VARIANTS[args.variant]
    traffic, traffic_src = pmc_traffic(variant, B, k, L, n)
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel": f"{KERNELS[variant]} (encode: {n} coded pieces x {B} objects per launch)",
        "kernel_ms": round(enc_ms, 4),
        "kernel_ms_how": ("HIP events around the encode launch on its stream, in pipeline-1 steps (the elimination "
                          "beside it, no other step's kernels)") if args.pipeline else "HIP events around the encode launch",
        "outputs_per_pass": n,
        "compulsory_bytes": enc_compulsory,
        "compulsory_GBps": round(enc_compulsory / (enc_ms * 1e-3) / 1e9, 1),
        "compulsory_frac": round(enc_compulsory / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "gf_muladd_per_s": round(ma_per_launch / (enc_ms * 1e-3) / 1e12, 3),
        "gf_muladd_unit": "T byte-multiply-adds/s",
    }

    # supplementary HBM roofline: the same source, ONE coded piece per object per launch (configs[1]'s encode
    # at one output row, ~1 multiply-add per source byte: the HBM-bound form of the north star's "encode at
    # k=32 x 1 MiB"); not part of `value`
    single = None
    if not args.encode_only:
        co1 = coeffs[:, :1].contiguous()
        out1 = torch.empty((B, 1, k + L), dtype=torch.uint8, device=dev)
        ts = []
        for r in range(12):
            a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch.encode_batch(src, co1, out1, ctx)
            b_.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(a.elapsed_time(b_))
        ms1 = sorted(ts)[len(ts) // 2]
        ok1 = torch.equal(out1[:, 0, k:], pieces[:, 0, k:])  # = coded piece 0 of the timed encode
        read1 = B * (k * L + k)
        single = {"coded_per_pass": 1, "kernel": "gf_matmul_stream_kernel<1, 2>", "ms": round(ms1, 4),
                  "source_read_GBps": round(read1 / ms1 / 1e6, 1),
                  "read_frac": round(read1 / ms1 / 1e6 / HBM_PEAK_GBS, 4),
                  "compulsory_GBps": round((read1 + B * (k + L)) / ms1 / 1e6, 1), "verified": bool(ok1)}

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: uniform random source bytes (torch generator, seeded per rank), coefficients "
                "uniform bytes from a seeded host RNG",
        "config": {
            "workload": f"per object: encode k={k} x {L} B -> {n} coded pieces (configs[1]) + decode from the "
                        f"first {m} (configs[2]); {B} objects per GPU per step",
            "k": k, "piece_bytes": L, "coded_per_object": n, "decoded_from": m, "objects_per_gpu": B,
            "parallelism": f"objects sharded over {dist.world} rank(s), no data-path collective",
            "kernel_variant": variant,
            "pipeline": {0: "serial", 1: "elimination on a side stream concurrent with the encode data work",
                         2: "elimination beside the encode data work, and step i+1's encode beside step i's decode "
                            "(two buffer sets)"}[args.pipeline],
        },
        "roofline": roofline,
        "hbm_single_pass_encode": single,
        "cpu_baseline": None,
        "breakdown": {
            "encode_kernel_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_GiBps_refcounter": round(B * n * encode_counter(k, L) / (enc_ms * 1e-3) / GIB, 1),
            "decode_GiBps_refcounter": round(B * decode_counter(k, L) / (dec_ms * 1e-3) / GIB, 2) if dec_ms else None,
            "roundtrip_goodput_GiBps": round(dist.world * B * k * L * args.steps / elapsed / GIB, 2),
            "verified": ok,
        },
    }
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(k, L, n, m, args.cpu_seconds)
        result["vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
        if args.cpu_threads > 1:  # the same on the box's CPU share (16 cores per GPU), one object per thread
            threads = min(args.cpu_threads, os.cpu_count() or 1)
            result["cpu_baseline_all_cores"] = cpu_baseline(k, L, n, m, args.cpu_seconds, threads)
            result["vs_cpu_baseline_all_cores"] = round(value / result["cpu_baseline_all_cores"]["value"], 1)
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()
    if not ok:
        print("VERIFICATION FAILED: decoded data does not match the source", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
