#!/usr/bin/env python3
"""The rocprofv3 durations of exactly the launches bench.py's rooflines time (roofline.kernel_ms, and with --decode
roofline_decode.kernel_ms).

bench.py (default --pipeline 2) runs --breakdown-steps + 6 launch groups of the pipeline-1 form BEFORE its warmup and
timed steps, and averages the HIP-event windows of all but the first 6.  Those are the first launches of the program
of the encode product (gf_matmul_bsj_kernel<8, true> at the encode grid) and of the decode's T x data product
(gf_matmul_bsj_kernel<4, true> at the decode grid: its 32-row tiles), so this selects launches [skip, skip + steps) of
that kernel at its most frequent grid, in start order, from the rocpd database of
`rocprofv3 --kernel-trace --stats -- python bench.py ...` and compares their average with the bench line of the same
run.  With --decode the decode apply's other launches in the same groups (its address launch and the marker scan) are
averaged too, so the product + them can be set against roofline_decode.kernel_ms (events around the whole apply).

    python3 scripts/breakdown_launches.py run_results.db bench.json [--steps 24 --skip 6] > profiles/rNN_....json
    python3 scripts/breakdown_launches.py run_results.db bench.json --decode > profiles/rNN_..._decode.json
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
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--decode", action="store_true", help="the decode product (roofline_decode) instead of the encode")
    a = ap.parse_args()
    kernel = a.kernel or ("gf_matmul_bsj_kernel<4, true>" if a.decode else "gf_matmul_bsj_kernel<8, true>")
    key = "roofline_decode" if a.decode else "roofline"
    line = json.loads([ln for ln in open(a.bench_json) if ln.startswith("{")][-1])
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, workgroup_x, start, duration from kernels order by start").fetchall()
    enc = [(gx, st, dur / 1e3) for name, gx, wx, st, dur in rows if kernel in name]
    grid = statistics.mode(gx for gx, _, _ in enc)  # the product's grid (not a probe launch's)
    launches = [(st, d) for gx, st, d in enc if gx == grid]
    enc = [d for _, d in launches]
    sel = enc[a.skip:a.skip + a.steps]
    avg = statistics.mean(sel)
    ma = line[key]["multiply_adds_per_launch"]
    extra = {}
    if a.decode:
        # the apply's other launches of the same groups: the address (offset) launch right before each selected
        # product on its stream and the marker scan right after it (first launch of each name after the product)
        picked = launches[a.skip:a.skip + a.steps]
        by_name = {}
        # the address launch counts only where it runs inside the window (bench.py --no-plan)
        names = ("bsj_offset_kernel", "final_len") if "bsj_offset_kernel" in line[key]["kernel"] else ("final_len",)
        for st0, d in picked:
            for name in names:
                cand = [(st, dur / 1e3) for nm, gx, wx, st, dur in rows if name in nm and
                        (st < st0 if name == "bsj_offset_kernel" else st > st0)]
                if cand:
                    by_name.setdefault(name, []).append(cand[-1][1] if name == "bsj_offset_kernel" else cand[0][1])
        extra = {f"{n}_avg_us": round(statistics.mean(v), 2) for n, v in by_name.items()}
        extra["product_plus_others_us"] = round(avg + sum(statistics.mean(v) for v in by_name.values()), 2)
        extra["kernel_ms_over_product_plus_others"] = round(line[key]["kernel_ms"] * 1e3 /
                                                            extra["product_plus_others_us"], 4)
    out = {
        "what": f"rocprofv3 kernel-trace durations of {kernel} (grid_x {grid}) launches {a.skip}..{a.skip + a.steps - 1} "
                f"in start order = bench.py's pipeline-1 breakdown groups (the launches {key}.kernel_ms averages)",
        "launches": len(sel),
        "avg_us": round(avg, 2),
        "median_us": round(statistics.median(sel), 2),
        "min_us": round(min(sel), 2),
        "max_us": round(max(sel), 2),
        "all_launches_avg_us": round(statistics.mean(enc), 2),
        "all_launches": len(enc),
        "bench_kernel_ms": line[key]["kernel_ms"],
        "kernel_ms_over_rocprof_avg": round(line[key]["kernel_ms"] * 1e3 / avg, 4),
        "achieved_T_ma_per_s_rocprof": round(ma / (avg * 1e-6) / 1e12, 2),
        "frac_rocprof": round(ma / (avg * 1e-6) / 1e12 / SPEC_PEAK_T_MA, 4),
        "bench_frac": line[key]["frac"],
        "peak": round(SPEC_PEAK_T_MA, 2),
        **extra,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
