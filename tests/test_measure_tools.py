"""CPU tests of the measurement tooling behind the bench line's rooflines (no device): scripts/breakdown_launches.py
selects, in a rocprofv3 kernel-trace database, exactly the launches bench.py's HIP events time (the pipeline-1 breakdown
groups before the timed loop: launches skip .. skip + steps - 1 of the product kernel at its most frequent grid), and
with --decode adds the decode apply's other launches inside the window; scripts/unit_breakdown.py turns the interleaved
diagnostic sweep into per-term costs."""
import json
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def make_db(path, with_offset):
    """Eight launch groups: (decode: offset) product, scan; encode product -- plus a probe launch at another grid."""
    c = sqlite3.connect(path)
    c.execute("create table kernels (name text, grid_x int, workgroup_x int, start int, duration int)")
    t = 0
    rows = [("void rlnc::gf_matmul_bsj_kernel<4, true>(...)", 256, 256, t, 1000)]  # probe-like, other grid
    t += 10_000
    for g in range(8):
        rows.append(("void rlnc::gf_matmul_bsj_kernel<8, true>(...)", 4194304, 512, t, 1_000_000 + 1000 * g))
        t += 1_100_000
        if with_offset:
            rows.append(("void rlnc::bsj_offset_kernel<true>(...)", 32768, 256, t, 5000))
            t += 6000
        rows.append(("void rlnc::gf_matmul_bsj_kernel<4, true>(...)", 2097152, 256, t, 500_000 + 1000 * g))
        t += 510_000
        rows.append(("void rlnc::final_len_scan_kernel<true>(...)", 512, 256, t, 4000))
        t += 5000
    c.executemany("insert into kernels values (?, ?, ?, ?, ?)", rows)
    c.commit()
    c.close()


def bench_line(path, with_offset):
    line = {"roofline": {"multiply_adds_per_launch": 1 << 36, "kernel_ms": 1.004, "frac": 0.2},
            "roofline_decode": {"multiply_adds_per_launch": 1 << 35, "kernel_ms": 0.510, "frac": 0.2,
                                "kernel": ("bsj_offset_kernel + " if with_offset else "") +
                                          "gf_matmul_bsj_kernel<4, true> + final_len_scan_kernel"}}
    with open(path, "w") as f:
        f.write("some log line\n" + json.dumps(line) + "\n")


def run(args):
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "breakdown_launches.py")] + args)
    return json.loads(out)


def test_breakdown_selects_the_timed_launches(tmp_path):
    db, bj = str(tmp_path / "run.db"), str(tmp_path / "b.json")
    make_db(db, with_offset=False)
    bench_line(bj, with_offset=False)
    enc = run([db, bj, "--steps", "4", "--skip", "2"])
    assert enc["launches"] == 4 and enc["all_launches"] == 8
    assert enc["avg_us"] == (1002 + 1003 + 1004 + 1005) / 4  # launches 2..5 in start order, us
    assert abs(enc["kernel_ms_over_rocprof_avg"] - 1.004 / 1.0035) < 1e-4
    dec = run([db, bj, "--steps", "4", "--skip", "2", "--decode"])
    assert dec["all_launches"] == 8  # the probe launch at another grid is not a product launch
    assert dec["avg_us"] == (502 + 503 + 504 + 505) / 4
    assert dec["final_len_avg_us"] == 4.0 and "bsj_offset_kernel_avg_us" not in dec  # written ahead: not in the window
    assert dec["product_plus_others_us"] == dec["avg_us"] + 4.0


def test_breakdown_counts_the_offset_launch_when_inside_the_window(tmp_path):
    db, bj = str(tmp_path / "run.db"), str(tmp_path / "b.json")
    make_db(db, with_offset=True)
    bench_line(bj, with_offset=True)  # bench.py --no-plan
    dec = run([db, bj, "--steps", "4", "--skip", "2", "--decode"])
    assert dec["bsj_offset_kernel_avg_us"] == 5.0 and dec["final_len_avg_us"] == 4.0
    assert dec["product_plus_others_us"] == dec["avg_us"] + 9.0


def test_unit_breakdown_terms(tmp_path):
    sweep = tmp_path / "sweep.txt"
    lines = []
    for rep in (1, 2):
        for name, enc in (("product", 1.2), ("s8inline", 1.08), ("s8nocombo", 1.05)):
            lines += [f"== {name} rep {rep}", json.dumps({"enc_ms_med": enc, "dec_ms_med": 0.6})]
    sweep.write_text("\n".join(lines) + "\n")
    out = json.loads(subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "unit_breakdown.py"),
                                              str(sweep)]))
    assert out["passes"] == 2 and out["product_enc_ms"] == 1.2
    assert abs(out["terms"]["s8inline"]["frac"] - 0.1) < 1e-9
    assert abs(out["terms"]["s8nocombo"]["frac"] - 0.125) < 1e-9
    # 2^36 / 4096 / 1024 units per SIMD at 2.15 GHz
    assert abs(out["simd_cycles_per_unit"] - round(1.2e-3 * 2.15e9 / 16384, 1)) < 1e-9
