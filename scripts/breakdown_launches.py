#!/usr/bin/env python3
"""The rocprofv3 durations of exactly the encode launches bench.py's roofline times (roofline.kernel_ms).

bench.py (default --pipeline 2) runs --breakdown-steps + 6 launch groups of the pipeline-1 form BEFORE its warmup and
timed steps, and averages the HIP-event encode windows of all but the first 6.  Those are the first encode launches of
the program (gf_matmul_bsj_kernel<8, true> at the encode grid), so this selects launches [skip, skip + steps) of that
kernel in start order from the rocpd database of `rocprofv3 --kernel-trace --stats -- python bench.py ...` and
compares their average with the bench line of the same run.

    python3 scripts/breakdown_launches.py run_results.db bench.json [--steps 24 --skip 6] > profiles/rNN_....json
"""
import argparse
import json
import sqlite3
import statistics

SPEC_PEAK_T_MA = 256 * 4 * 2.4e9 / 2 * 256 / 1e12  # bench.SPEC_PEAK_T_MA (the guide's VALU issue rate x 256)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("bench_json", help="the bench line of the profiled run (one JSON object)")
    ap.add_argument("--steps", type=int, default=24, help="bench.py --breakdown-steps")
    ap.add_argument("--skip", type=int, default=6)
    ap.add_argument("--kernel", default="gf_matmul_bsj_kernel<8, true>")
    a = ap.parse_args()
    line = json.loads([ln for ln in open(a.bench_json) if ln.startswith("{")][-1])
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, workgroup_x, start, duration from kernels order by start").fetchall()
    enc = [(gx, wx, dur / 1e3) for name, gx, wx, st, dur in rows if a.kernel in name]
    grid = enc[0][0]  # the first launch of the kernel is a breakdown group's encode
    enc = [d for gx, wx, d in enc if gx == grid]
    sel = enc[a.skip:a.skip + a.steps]
    avg = statistics.mean(sel)
    ma = line["roofline"]["multiply_adds_per_launch"]
    out = {
        "what": f"rocprofv3 kernel-trace durations of {a.kernel} (grid_x {grid}) launches {a.skip}..{a.skip + a.steps - 1} "
                "in start order = bench.py's pipeline-1 breakdown groups (the launches roofline.kernel_ms averages)",
        "launches": len(sel),
        "avg_us": round(avg, 2),
        "median_us": round(statistics.median(sel), 2),
        "min_us": round(min(sel), 2),
        "max_us": round(max(sel), 2),
        "all_encode_launches_avg_us": round(statistics.mean(enc), 2),
        "all_encode_launches": len(enc),
        "bench_kernel_ms": line["roofline"]["kernel_ms"],
        "kernel_ms_over_rocprof_avg": round(line["roofline"]["kernel_ms"] * 1e3 / avg, 4),
        "achieved_T_ma_per_s_rocprof": round(ma / (avg * 1e-6) / 1e12, 2),
        "frac_rocprof": round(ma / (avg * 1e-6) / 1e12 / SPEC_PEAK_T_MA, 4),
        "bench_frac": line["roofline"]["frac"],
        "peak": round(SPEC_PEAK_T_MA, 2),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
