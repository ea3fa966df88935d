#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

Run from the repo root in the build container:  python tests/golden/make_golden.py

1. gf256_tables.json — the reference's literal GF256_LOG_TABLE / GF256_EXP_TABLE values, parsed as data
   from /root/reference/src/common/gf256.rs:16-44 (only when that file is present; the committed JSON is
   what the tests use, so the GPU box never needs the reference).
2. vectors.json — encode / recode / incremental-decode / marker-trim / rref vectors at small sizes.  Each
   vector is produced by the C oracle (oracle/liboracle.so) AND by the independent numpy restatement
   (oracle/np_oracle.py, Russian-peasant field multiply), and is only written if both agree byte-for-byte.

The reference's own tests carry no known-answer vectors for coding outputs (all use OS-seeded rand::rng(),
SURVEY.md §4), so these fixtures are pinned by: the literal tables, FIPS-197 field products, the reference's
deterministic tests (swap_rows KAT decoder_matrix.rs:326-381, getter arithmetic encoder.rs:497-544) and two
independent restatements agreeing.
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import np_oracle as npo  # noqa: E402
from oracle.oracle import Oracle, OracleDecoder  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF_GF256 = "/root/reference/src/common/gf256.rs"

STATUS = ["Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
          "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful",
          "ReceivedAllPieces", "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength",
          "InvalidOutputBuffer"]


def hx(a) -> str:
    return np.asarray(a, np.uint8).tobytes().hex()


def extract_tables():
    if not os.path.exists(REF_GF256):
        print("reference not present; keeping committed gf256_tables.json")
        return
    txt = open(REF_GF256).read()

    def arr(name):
        m = re.search(name + r": \[u8; [^\]]*\] = \[(.*?)\];", txt, re.S)
        return [int(x) for x in re.findall(r"\d+", m.group(1))]

    log = arr("GF256_LOG_TABLE")
    exp = arr("GF256_EXP_TABLE")
    assert len(log) == 256 and len(exp) == 510
    with open(os.path.join(HERE, "gf256_tables.json"), "w") as f:
        json.dump({"source": "src/common/gf256.rs:16-44 (itzmeanjan/rlnc 0.8.5), literal values",
                   "log": log, "exp": exp}, f)
    print("wrote gf256_tables.json")


def coeff_rows(rng, n, k, special=True):
    c = rng.integers(0, 256, size=(n, k), dtype=np.uint8)
    if special and n >= 3:
        c[0, :] = 1          # c==1 fast path (simd/mod.rs:96-99)
        c[1, ::2] = 0        # c==0 early-out (simd/mod.rs:93-95)
        c[2, 1::2] = 1
    return c


def main():
    extract_tables()
    orc = Oracle()
    rng = np.random.default_rng(0x524C4E43)
    out = {"status_names": STATUS}

    # ---- encode ------------------------------------------------------------------------------
    enc = []
    for (k, L, n) in [(1, 1, 2), (1, 2, 3), (2, 15, 4), (4, 16, 5), (16, 17, 6), (3, 1000, 4), (32, 4096, 8),
                      (5, 33, 3)]:
        src = rng.integers(0, 256, size=(k, L), dtype=np.uint8)
        co = coeff_rows(rng, n, k)
        a = orc.encode(src, co)
        b = npo.encode(src, co)
        assert np.array_equal(a, b), (k, L)
        enc.append({"k": k, "L": L, "n": n, "src": hx(src), "coeffs": hx(co), "out": hx(a)})
    out["encode"] = enc

    # ---- padding (Encoder::new) -------------------------------------------------------------------
    pads = []
    for (dlen, k) in [(1, 1), (10, 10), (100, 50), (100, 1), (1023, 32), (1024, 32), (31, 32), (32, 32), (33, 32)]:
        data = rng.integers(0, 256, size=dlen, dtype=np.uint8)
        a = orc.pad(data, k)
        b = npo.pad(data, k)
        assert np.array_equal(a, b)
        pads.append({"data": hx(data), "k": k, "L": int(a.shape[1]), "padded": hx(a)})
    out["pad"] = pads

    # ---- recode --------------------------------------------------------------------------------
    rec = []
    for (k, L, nrecv) in [(4, 16, 3), (8, 64, 8), (16, 100, 5), (2, 1, 2)]:
        src = rng.integers(0, 256, size=(k, L), dtype=np.uint8)
        pieces = orc.encode(src, coeff_rows(rng, nrecv, k, special=False))
        r = rng.integers(0, 256, size=nrecv, dtype=np.uint8)
        r[0] = 1
        a = orc.recode(pieces, k + L, k, r)
        b = npo.recode(pieces, k, r)
        assert np.array_equal(a, b)
        rec.append({"k": k, "L": L, "n": nrecv, "pieces": hx(pieces), "r": hx(r), "out": hx(a)})
    out["recode"] = rec

    # ---- incremental decode sequences -------------------------------------------------------------
    dec = []

    def run_seq(name, k, L, pieces):
        od = OracleDecoder(L, k)
        nd = npo.Decoder(L, k)
        sts = []
        for p in pieces:
            s1 = STATUS[od.decode(p)]
            s2 = nd.decode(p)
            assert s1 == s2, (name, s1, s2)
            sts.append(s1)
        pay = od.padded_payload()
        assert np.array_equal(pay, nd.padded_payload()), name
        st, data = od.get_decoded_data()
        ent = {"name": name, "k": k, "L": L, "pieces": [hx(p) for p in pieces], "statuses": sts,
               "rows": int(pay.shape[0]), "payload": hx(pay), "final_status": STATUS[st],
               "data": hx(data) if st == 0 else None}
        dec.append(ent)

    # dense round trips with duplicates / recoded (useless) pieces interleaved
    for (dlen, k) in [(100, 4), (1000, 16), (64, 32), (5000, 8)]:
        data = rng.integers(0, 256, size=dlen, dtype=np.uint8)
        src = orc.pad(data, k)
        L = src.shape[1]
        coded = orc.encode(src, rng.integers(0, 256, size=(k + 4, k), dtype=np.uint8))
        seq = [coded[0], coded[0].copy(), coded[1]]
        seq.append(orc.recode(np.stack(seq[:3]), k + L, k, np.array([3, 7, 9], np.uint8)))  # dependent
        seq += list(coded[2:])
        run_seq(f"dense_d{dlen}_k{k}", k, L, seq)
        # the decoded data must round-trip
        assert dec[-1]["data"] == hx(data), dec[-1]["name"]
    # structured/sparse coefficients: diagonal-pivot quirk
    k, L = 6, 3
    vecs = [[0, 0, 2, 0, 0, 3], [0, 0, 0, 2, 2, 0], [0, 0, 0, 0, 0, 2], [0, 0, 0, 0, 0, 1]]
    pieces = [np.concatenate([np.array(v, np.uint8), rng.integers(0, 256, size=L, dtype=np.uint8)]) for v in vecs]
    run_seq("overcount_k6", k, L, pieces)
    # sparse random pieces, many zero coefficients
    for trial in range(6):
        k, L = 8, 5
        ps = []
        for _ in range(14):
            cv = rng.integers(0, 256, size=k, dtype=np.uint8)
            cv[rng.random(k) < 0.7] = 0
            ps.append(np.concatenate([cv, rng.integers(0, 256, size=L, dtype=np.uint8)]))
        run_seq(f"sparse_{trial}", k, L, ps)
    # identity (systematic) pieces in reverse order, then extra
    k, L = 5, 7
    data = rng.integers(0, 256, size=30, dtype=np.uint8)
    src = orc.pad(data, k)
    eye = np.eye(k, dtype=np.uint8)[::-1]
    run_seq("systematic_reverse", k, src.shape[1], list(orc.encode(src, eye)) + [orc.encode(src, eye[:1])[0]])
    # wrong-length piece, then a valid sequence (state must not change on invalid input, decoder.rs:266-269)
    k, L = 3, 4
    src = orc.pad(rng.integers(0, 256, size=9, dtype=np.uint8), k)
    cod = orc.encode(src, rng.integers(1, 256, size=(4, k), dtype=np.uint8))
    run_seq("invalid_len_first", k, src.shape[1], [cod[0][:-1], np.zeros(0, np.uint8)] + list(cod))
    out["decode"] = dec

    # ---- final_data_len edge cases (decoder.rs:162-177) -----------------------------------------------
    fdl = []
    cases = [[0x81], [1, 0x81], [1, 0x81, 0], [1, 0x81, 0, 0], [0x81, 0, 0], [1, 2, 3], [0, 0, 0],
             [1, 0x81, 5], [1, 0x81, 0x81], [1, 0x81, 0x81, 0], [7, 0x81, 0, 0x81, 0], [0x81, 0x81]]
    for c in cases:
        a = np.array(c, np.uint8)
        st, n = orc.final_data_len(a)
        ok, n2 = npo.final_data_len(a)
        assert (st == 0) == ok and (not ok or n == n2), c
        fdl.append({"padded": hx(a), "status": STATUS[st], "len": n if st == 0 else None})
    out["final_data_len"] = fdl

    # ---- rref of random / structured matrices --------------------------------------------------------
    rr = []
    for (rows, cols, k, density) in [(4, 5, 3, 1.0), (6, 6, 6, 0.5), (10, 7, 7, 0.3), (3, 12, 3, 1.0),
                                     (12, 12, 4, 0.4), (1, 1, 1, 1.0), (5, 9, 9, 0.2)]:
        m = rng.integers(0, 256, size=(rows, cols), dtype=np.uint8)
        m[rng.random((rows, cols)) > density] = 0
        a = orc.rref(m, k)
        b = npo.rref(m, k)
        assert np.array_equal(a, b)
        assert np.array_equal(orc.rref(a, k), a)  # decoder_matrix.rs:303-324 idempotence
        rr.append({"rows": rows, "cols": cols, "k": k, "in": hx(m), "out_rows": int(a.shape[0]), "out": hx(a)})
    out["rref"] = rr

    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote vectors.json", os.path.getsize(os.path.join(HERE, "vectors.json")), "bytes")


if __name__ == "__main__":
    main()
