#!/usr/bin/env python3
"""Host-resident rate of the library's own streaming API.

Same per-object workload as bench.py (encode k=32 × 1 MiB → 64 coded pieces, decode from the first 32), but every
object starts and ends in host memory and crosses PCIe through librlnc_hip's pipeline:
    rlnc_encode_host_stream: source (host) → 64 coded pieces (host)
    rlnc_decode_host_stream: the first 32 coded pieces of each object (host, strided) → decoded rows (host)
once with pinned host buffers (DMA straight from/to them) and once with pageable ones (staged through the
library's pinned buffers by host threads), each call after the other ("serial"); then, as an endpoint that both sends
and receives does it, the encode of step i and the decode of step i-1 as two concurrent calls from two host threads
on two contexts (pinned, "concurrent": two buffer sets, so both PCIe directions carry traffic at once).  Reports GiB/s in bench.py's counters, the PCIe bytes moved, the raw
pinned copy rates of the box, and checks decoded == source for every object.
"""
# HIP multiplexes streams over GPU_MAX_HW_QUEUES hardware queues (4 by default); the library's pipeline keeps three
# streams busy (compute, host->device, device->host), and with 4 queues a copy stream can share a queue with another
# stage of this process.  Run it as `GPU_MAX_HW_QUEUES=16 python scripts/host_stream_rate.py` to give every stream
# its own queue (profiles/r02_host_stream_ab.txt has both); the value in use is reported.
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bind_to_gpu_node(dev=0):
    """Pin this process's threads to the CPUs of the GPU's NUMA node (the pinned host buffers are then first-touched
    there, so PCIe traffic does not cross the socket interconnect).  Returns the node, or None if unknown."""
    import torch

    try:
        pr = torch.cuda.get_device_properties(dev)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    except Exception:
        return None
    try:
        node = int(open(f"/sys/bus/pci/devices/{bus.lower()}/numa_node").read())
        if node < 0:
            return None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return node
    except OSError:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--window", type=int, default=0, help="objects per pipeline window (0 = library default)")
    ap.add_argument("--no-numa-bind", action="store_true", help="do not pin the process to the GPU's NUMA node")
    ap.add_argument("--modes", default="pinned,pageable,concurrent,raw",
                    help="comma list of pinned, pageable, concurrent, raw (the box's raw copy rates)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import rlnc_amd

    k, L, n, m, B = 32, 1 << 20, 64, 32, args.objects
    node = None if args.no_numa_bind else bind_to_gpu_node(0)
    ctx = rlnc_amd.Context(0)
    lib = ctx.lib
    rng = np.random.default_rng(1)
    out = {"metric": "host-resident RLNC encode+decode GiB/s (library pipeline, host buffers in and out), "
                     "k=32 x 1 MiB", "unit": "GiB/s", "objects": B,
           "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
           "numa_node_bound": node, "cpus": len(os.sched_getaffinity(0))}
    modes = set(args.modes.split(","))
    for mode in [x for x in ("pinned", "pageable") if x in modes]:
        pin = mode == "pinned"

        def buf(shape):
            return torch.empty(shape, dtype=torch.uint8, pin_memory=pin)

        src, co, pieces, dec = buf((B, k, L)), buf((B, n, k)), buf((B, n, k + L)), buf((B, k, L))
        src.numpy()[...] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        co.numpy()[...] = rng.integers(0, 256, (B, n, k), dtype=np.uint8)
        ps = np.zeros((B, m), np.int32)
        os_ = np.zeros(B, np.int32)
        dl = np.zeros(B, np.uint64)
        p = lambda t: C.c_void_p(t.data_ptr())

        part = {"encode": 0.0, "decode": 0.0}

        def step():
            t = time.perf_counter()
            assert lib.rlnc_encode_host_stream(ctx.h, p(src), k, L, B, p(co), n, p(pieces), args.window) == 0
            t2 = time.perf_counter()
            assert lib.rlnc_decode_host_stream(ctx.h, p(pieces), n * (k + L), k, L, m, B, p(dec),
                                               ps.ctypes.data_as(C.POINTER(C.c_int32)),
                                               os_.ctypes.data_as(C.POINTER(C.c_int32)),
                                               dl.ctypes.data_as(C.POINTER(C.c_uint64)), args.window) == 0
            part["encode"] += t2 - t
            part["decode"] += time.perf_counter() - t2

        step()  # warm-up: the library's pipeline buffers are allocated once and kept
        part["encode"] = part["decode"] = 0.0
        t0 = time.perf_counter()
        per_step = []
        for _ in range(args.steps):
            ts = time.perf_counter()
            step()
            per_step.append(round((time.perf_counter() - ts) * 1e3, 2))
        el = (time.perf_counter() - t0) / args.steps
        ok = all((ps[o] == 0).sum() < k or np.array_equal(dec.numpy()[o], src.numpy()[o]) for o in range(B))
        moved = B * (k * L + n * k + n * (k + L) + m * (k + L) + k * L)
        out[mode] = {"value": round(bench.step_bytes(B, k, L, n) / el / 2**30, 2), "ms_per_step": round(el * 1e3, 2),
                     "pcie_bytes_per_step": moved, "pcie_GBps_effective": round(moved / el / 1e9, 2),
                     "roundtrip_goodput_GiBps": round(B * k * L / el / 2**30, 3), "verified": bool(ok),
                     "encode_call_ms": round(part["encode"] / args.steps * 1e3, 2),
                     "encode_call_GBps": round(B * (k * L + n * k + n * (k + L)) / (part["encode"] / args.steps) / 1e9, 2),
                     "decode_call_ms": round(part["decode"] / args.steps * 1e3, 2),
                     "decode_call_GBps": round(B * (m * (k + L) + k * L) / (part["decode"] / args.steps) / 1e9, 2),
                     "step_ms": per_step}
        del src, co, pieces, dec
    # concurrent: step i's encode (thread A, context A) beside step i-1's decode (thread B, context B); ctypes releases
    # the GIL inside the library, so the two calls overlap on the device and on PCIe
    import threading

    if "concurrent" not in modes:
        print(json.dumps(out), flush=True)
        return
    ctx2 = rlnc_amd.Context(0)
    buf = lambda shape: torch.empty(shape, dtype=torch.uint8, pin_memory=True)
    src, co = buf((B, k, L)), buf((B, n, k))
    src.numpy()[...] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    co.numpy()[...] = rng.integers(0, 256, (B, n, k), dtype=np.uint8)
    pieces = [buf((B, n, k + L)), buf((B, n, k + L))]
    dec = buf((B, k, L))
    ps = np.zeros((B, m), np.int32)
    os_ = np.zeros(B, np.int32)
    dl = np.zeros(B, np.uint64)
    p = lambda t: C.c_void_p(t.data_ptr())
    rcs = {}

    def enc(i):
        rcs["e"] = lib.rlnc_encode_host_stream(ctx.h, p(src), k, L, B, p(co), n, p(pieces[i % 2]), args.window)

    def decd(i):
        rcs["d"] = lib.rlnc_decode_host_stream(ctx2.h, p(pieces[(i - 1) % 2]), n * (k + L), k, L, m, B, p(dec),
                                               ps.ctypes.data_as(C.POINTER(C.c_int32)),
                                               os_.ctypes.data_as(C.POINTER(C.c_int32)),
                                               dl.ctypes.data_as(C.POINTER(C.c_uint64)), args.window)

    def cstep(i):
        ts = [threading.Thread(target=enc, args=(i,))] + ([threading.Thread(target=decd, args=(i,))] if i else [])
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert all(v == 0 for v in rcs.values()), rcs

    cstep(0)
    cstep(1)  # warm-up: both contexts' pipeline buffers allocated
    t0 = time.perf_counter()
    for i in range(2, 2 + args.steps):
        cstep(i)
    el = (time.perf_counter() - t0) / args.steps
    ok = all((ps[o] == 0).sum() < k or np.array_equal(dec.numpy()[o], src.numpy()[o]) for o in range(B))
    moved = B * (k * L + n * k + n * (k + L) + m * (k + L) + k * L)
    out["concurrent"] = {"value": round(bench.step_bytes(B, k, L, n) / el / 2**30, 2), "ms_per_step": round(el * 1e3, 2),
                         "pcie_bytes_per_step": moved, "pcie_GBps_effective": round(moved / el / 1e9, 2),
                         "roundtrip_goodput_GiBps": round(B * k * L / el / 2**30, 3), "verified": bool(ok),
                         "how": "encode of step i and decode of step i-1 from two host threads on two contexts"}
    del src, co, pieces, dec
    # the bidirectional ceiling: 1 GiB host->device and 1 GiB device->host at once on two streams
    h_a = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    h_b = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    d_b = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for it in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            d_a.copy_(h_a, non_blocking=True)
        with torch.cuda.stream(s2):
            h_b.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    out["pinned_bidirectional_GBps"] = round(2 * (1 << 30) / el / 1e9, 2)
    for mode in ("pinned", "pageable", "concurrent"):
        if mode in out:
            out[mode]["frac_of_bidirectional"] = round(out[mode]["pcie_GBps_effective"] / out["pinned_bidirectional_GBps"], 4)
    del h_a, h_b, d_a, d_b
    # raw pinned copy rates of this box
    big_h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    big_d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    t = time.perf_counter()
    big_d.copy_(big_h, non_blocking=True)
    torch.cuda.synchronize()
    out["pinned_h2d_GBps"] = round((1 << 30) / (time.perf_counter() - t) / 1e9, 2)
    t = time.perf_counter()
    big_h.copy_(big_d, non_blocking=True)
    torch.cuda.synchronize()
    out["pinned_d2h_GBps"] = round((1 << 30) / (time.perf_counter() - t) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
