#!/usr/bin/env python3
"""Per-term breakdown of the 8-wave encode unit from scripts/archive/r06_unit_breakdown.sh's interleaved sweep
(gen_bsjump.py --diag=s8* timing-only builds against the product library).  Each term = the product's median encode
launch time minus the build without that term (mean over the passes), as a fraction of the product's time and as SIMD
cycles per (row, source, wave) unit: 2^36 multiply-adds per launch / 4,096 per unit / 1,024 SIMDs = 16,384 units per
SIMD, at the clock given (--ghz, the PMC-measured 2.15 under this load).

    python3 scripts/unit_breakdown.py profiles/r06_unit_breakdown_sweep.txt > profiles/r06_unit_breakdown.json
"""
import argparse
import collections
import json

TERMS = {
    "s8inline": "calls: s_swappc + the block's s_setpc per (row, source), the block inlined (relative XOR3s kept)",
    "s8noread": "set reads: 16 ds_read_b128 per wave per source row (4 with set planes; registers left stale)",
    "s8noown": "set building: the builders' half transpose + 11 composite XORs (set writes kept)",
    "s8nosmem": "address stream: s_load_dwordx16 of the next row's 8 block addresses",
    "s8nobar": "barrier: s_barrier every third source row",
    "s8nodma": "LDS-DMA of source rows (global_load_lds_dwordx4)",
    "s8nostage": "staging reads of the next source row from the LDS ring",
    "s8nocombo": "composites: the 44 VOP2 XORs per source row and wave that build the sets from their planes (set "
                 "planes form, round 6)",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep")
    ap.add_argument("--ghz", type=float, default=2.15)
    a = ap.parse_args()
    runs = collections.defaultdict(list)
    cur = None
    for ln in open(a.sweep):
        if ln.startswith("=="):
            cur = ln.split()[1]
        elif ln.startswith("{") and cur:
            runs[cur].append(json.loads(ln))
    prod = sum(r["enc_ms_med"] for r in runs["product"]) / len(runs["product"])
    units = (1 << 36) / 4096 / 1024
    cyc = prod * 1e-3 * a.ghz * 1e9 / units
    out = {"what": "8-wave encode unit (gf_matmul_bsj_kernel<8, true>, bench shape), per-term cost by removal",
           "product_enc_ms": round(prod, 4), "passes": len(runs["product"]), "ghz": a.ghz,
           "simd_cycles_per_unit": round(cyc, 1), "terms": {}}
    for name, what in TERMS.items():
        if name not in runs:
            continue
        t = sum(r["enc_ms_med"] for r in runs[name]) / len(runs[name])
        d = prod - t
        out["terms"][name] = {"what": what, "enc_ms": round(t, 4), "saved_ms": round(d, 4),
                              "frac": round(d / prod, 4), "cycles_per_unit": round(d / prod * cyc, 1),
                              "dec_ms_control": round(sum(r["dec_ms_med"] for r in runs[name]) / len(runs[name]), 4)}
    out["rest_cycles_per_unit"] = round(cyc - sum(max(0.0, v["cycles_per_unit"]) for v in out["terms"].values()), 1)
    out["rest_note"] = ("what no single removal accounts for: the 16 GPR-index-relative XOR3s of each call (77 SIMD "
                        "cycles inline per profiles/r02_ubench_tables.jsonl) and overlap between the terms")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
