"""CPU: pin the oracle (C restatement + numpy restatement) against everything the reference fixes.

The reference (Rust) cannot run here, so the pins are: its literal field tables (gf256.rs:16-44),
FIPS-197 AES-field KATs, its deterministic tests (swap_rows KAT decoder_matrix.rs:326-381, getter
arithmetic encoder.rs:497-544, error-order tables in every module's tests) and its property tests
(gf256.rs:188-215, decoder_matrix.rs:303-324, full/tests.rs:7-203), re-run on the oracle.
"""
import numpy as np
import pytest

from oracle import np_oracle as npo
from oracle.oracle import OracleDecoder
from tests.conftest import hexarr

S = ["Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
     "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful", "ReceivedAllPieces",
     "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength", "InvalidOutputBuffer"]


def test_tables_match_reference_literals(orc, ref_tables):
    log, exp = orc.tables()
    assert list(log) == ref_tables["log"]
    assert list(exp) == ref_tables["exp"]


def test_fips197_kats(orc):
    # FIPS-197 §4.2: {57}·{83} = {c1}; §4.2.1: {57}·{13} = {fe}, xtime({57}) = {ae}; §5.1.1: {53}^-1 = {ca}
    assert orc.mul(0x57, 0x83) == 0xC1
    assert orc.mul(0x57, 0x13) == 0xFE
    assert orc.mul(0x57, 0x02) == 0xAE
    assert orc.inv(0x53) == 0xCA
    assert orc.inv(0) is None


def test_full_product_table_two_restatements(orc):
    assert np.array_equal(orc.mul_table(), npo.mul_table())


def test_nibble_split_identity(orc):
    # simd_mul_table.rs:36-80: c·x = LOW[c][x & 15] ^ HIGH[c][x >> 4], bytes 16..31 zero
    low, high = orc.nibble_tables()
    x = np.arange(256)
    M = npo.mul_table()
    for c in range(256):
        assert np.array_equal(low[c][x & 15] ^ high[c][x >> 4], M[c])
    assert not low[:, 16:].any() and not high[:, 16:].any()


def test_field_properties(orc):
    # gf256.rs:188-215
    rng = np.random.default_rng(1)
    for a, b in rng.integers(0, 256, size=(20000, 2)):
        a, b = int(a), int(b)
        assert ((a ^ b) ^ b) == a
        prod = orc.mul(a, b)
        if b == 0:
            assert prod == 0 and orc.inv(b) is None
        else:
            assert orc.mul(prod, orc.inv(b)) == a


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 1000, 4099])
def test_vector_primitives_simd_vs_scalar(orc, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    for c in [0, 1, 2, 0x53, 0xFF]:
        fast = (orc.mul_vec_by_scalar(a, c), orc.mul_add(b, a, c), orc.add_vectors(b, a))
        orc.force_scalar(True)
        try:
            slow = (orc.mul_vec_by_scalar(a, c), orc.mul_add(b, a, c), orc.add_vectors(b, a))
        finally:
            orc.force_scalar(False)
        M = npo.mul_table()
        assert np.array_equal(fast[0], M[c][a]) and np.array_equal(slow[0], fast[0])
        assert np.array_equal(fast[1], b ^ M[c][a]) and np.array_equal(slow[1], fast[1])
        assert np.array_equal(fast[2], a ^ b) and np.array_equal(slow[2], fast[2])


def test_golden_encode(orc, golden):
    for v in golden["encode"]:
        k, L = v["k"], v["L"]
        src = hexarr(v["src"]).reshape(k, L)
        co = hexarr(v["coeffs"]).reshape(v["n"], k)
        assert orc.encode(src, co).tobytes().hex() == v["out"]


def test_golden_pad(orc, golden):
    for v in golden["pad"]:
        a = orc.pad(hexarr(v["data"]), v["k"])
        assert a.shape[1] == v["L"] and a.tobytes().hex() == v["padded"]


def test_golden_recode(orc, golden):
    for v in golden["recode"]:
        k, L, n = v["k"], v["L"], v["n"]
        out = orc.recode(hexarr(v["pieces"]).reshape(n, k + L), k + L, k, hexarr(v["r"]))
        assert out.tobytes().hex() == v["out"]


def test_golden_decode_sequences(golden):
    for v in golden["decode"]:
        d = OracleDecoder(v["L"], v["k"])
        sts = [S[d.decode(hexarr(p))] for p in v["pieces"]]
        assert sts == v["statuses"], v["name"]
        assert d.padded_payload().tobytes().hex() == v["payload"], v["name"]
        st, data = d.get_decoded_data()
        assert S[st] == v["final_status"], v["name"]
        if st == 0:
            assert data.tobytes().hex() == v["data"]


def test_overcount_quirk_is_replicated(golden):
    # the diagonal-pivot RREF reports rank 4 for 4 vectors of true rank 3
    v = [x for x in golden["decode"] if x["name"] == "overcount_k6"][0]
    assert v["statuses"] == ["Ok"] * 4 and v["rows"] == 4
    M = np.stack([hexarr(p)[:6] for p in v["pieces"]])
    assert true_rank(M) == 3  # rows 2 and 3 are dependent
    assert npo.rref(M, 6).shape[0] == 4  # the reference algorithm still says 4


def true_rank(M):
    """Textbook rank over GF(2^8) (pivot search in every column) — NOT the reference's algorithm."""
    M = np.array(M, np.uint8)
    T = npo.mul_table()
    r = 0
    for c in range(M.shape[1]):
        piv = [i for i in range(r, M.shape[0]) if M[i, c]]
        if not piv:
            continue
        M[[r, piv[0]]] = M[[piv[0], r]]
        inv = npo.gf_inv(int(M[r, c]))
        M[r] = T[inv][M[r]]
        for i in range(M.shape[0]):
            if i != r and M[i, c]:
                M[i] ^= T[int(M[i, c])][M[r]]
        r += 1
    return r


def test_golden_final_data_len(orc, golden):
    for v in golden["final_data_len"]:
        st, n = orc.final_data_len(hexarr(v["padded"]))
        assert S[st] == v["status"]
        if st == 0:
            assert n == v["len"]


def test_golden_rref_and_idempotence(orc, golden):
    for v in golden["rref"]:
        m = hexarr(v["in"]).reshape(v["rows"], v["cols"])
        r = orc.rref(m, v["k"])
        assert r.shape[0] == v["out_rows"] and r.tobytes().hex() == v["out"]
        assert np.array_equal(orc.rref(r, v["k"]), r)


def test_rref_idempotent_random(orc):
    # decoder_matrix.rs:303-324 (sizes reduced)
    rng = np.random.default_rng(7)
    for _ in range(60):
        rows, cols = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        m = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
        a = orc.rref(m, cols)
        assert np.array_equal(orc.rref(a, cols), a)
        assert np.array_equal(a, npo.rref(m, cols))


def test_swap_rows_kat(orc):
    # decoder_matrix.rs:326-381
    m = np.array([[1, 1, 1, 10, 10], [2, 2, 2, 20, 20], [3, 3, 3, 30, 30], [4, 4, 4, 40, 40]], np.uint8)
    assert orc.swap_rows(m, 0, 2).tolist() == [[3, 3, 3, 30, 30], [2, 2, 2, 20, 20], [1, 1, 1, 10, 10], [4, 4, 4, 40, 40]]
    assert orc.swap_rows(m, 3, 1).tolist() == [[1, 1, 1, 10, 10], [4, 4, 4, 40, 40], [3, 3, 3, 30, 30], [2, 2, 2, 20, 20]]
    assert orc.swap_rows(m, 1, 1).tolist() == m.tolist()
    assert orc.swap_rows(m, 0, 3).tolist() == [[4, 4, 4, 40, 40], [2, 2, 2, 20, 20], [3, 3, 3, 30, 30], [1, 1, 1, 10, 10]]


def test_getter_arithmetic(orc):
    # encoder.rs:497-544
    assert orc.piece_byte_len(100, 1) == 101
    assert orc.piece_byte_len(1, 1) == 2 and 1 + orc.piece_byte_len(1, 1) == 3
    assert orc.piece_byte_len(10, 10) == 2
    assert orc.piece_byte_len(100, 50) == (100 + 1 + 49) // 50


def test_error_orders(orc):
    lib = orc.lib
    import ctypes as C

    buf = np.zeros(16, np.uint8)
    p = buf.ctypes.data_as(C.POINTER(C.c_uint8))
    assert S[lib.orc_encoder_pad(p, 0, 0, p)] == "DataLengthZero"  # encoder.rs:339-349
    assert S[lib.orc_encoder_pad(p, 5, 0, p)] == "PieceCountZero"
    src = np.zeros((4, 4), np.uint8)
    assert S[orc.code_with_coding_vector(src, np.zeros(3, np.uint8))[0]] == "CodingVectorLengthMismatch"
    assert S[orc.code_with_coding_vector(src, np.zeros(4, np.uint8), out_len=3)[0]] == "InvalidOutputBuffer"
    assert S[orc.code_with_coding_vector(src, np.zeros(0, np.uint8), out_len=8)[0]] == "CodingVectorLengthMismatch"
    r = np.zeros(1, np.uint8)
    rp = r.ctypes.data_as(C.POINTER(C.c_uint8))
    o = np.zeros(64, np.uint8)
    op = o.ctypes.data_as(C.POINTER(C.c_uint8))
    f = lib.orc_recode_with_vector
    assert S[f(p, 0, 8, 4, rp, 1, op, 8)] == "NotEnoughPiecesToRecode"  # recoder.rs:191-240
    assert S[f(p, 3, 0, 4, rp, 1, op, 0)] == "PieceLengthZero"
    assert S[f(p, 3, 8, 0, rp, 1, op, 8)] == "PieceCountZero"
    assert S[f(p, 3, 4, 4, rp, 1, op, 4)] == "PieceLengthTooShort"
    assert S[f(p, 3, 3, 4, rp, 1, op, 3)] == "PieceLengthTooShort"
    st = C.c_int(0)
    assert lib.orc_decoder_new(0, 10, C.byref(st)) is None and S[st.value] == "PieceLengthZero"  # decoder.rs:187-220
    assert lib.orc_decoder_new(10, 0, C.byref(st)) is None and S[st.value] == "PieceCountZero"
    assert lib.orc_decoder_new(0, 0, C.byref(st)) is None and S[st.value] == "PieceLengthZero"


def test_decoder_invalid_length_keeps_state():
    # decoder.rs:222-287
    d = OracleDecoder(4, 3)
    assert S[d.decode(np.zeros(6, np.uint8))] == "InvalidPieceLength"
    assert S[d.decode(np.zeros(8, np.uint8))] == "InvalidPieceLength"
    assert S[d.decode(np.zeros(0, np.uint8))] == "InvalidPieceLength"
    assert d.received == 0 and d.useful == 0 and not d.is_already_decoded()


@pytest.mark.parametrize("seed", range(3))
def test_roundtrip_properties(orc, seed):
    # full/tests.rs:7-203 (sizes reduced so the CPU suite stays fast)
    rng = np.random.default_rng(100 + seed)
    dlen = int(rng.integers(1 << 10, 1 << 14))
    k = int(rng.integers(8, 48))
    data = rng.integers(0, 256, dlen, dtype=np.uint8)
    src = orc.pad(data, k)
    L = src.shape[1]
    dec = OracleDecoder(L, k)
    seen = []
    for _ in range(k // 2):
        p = orc.encode(src, rng.integers(0, 256, (1, k), dtype=np.uint8))[0]
        if S[dec.decode(p)] == "Ok":
            seen.append(p)
    # recoded combinations of already-seen pieces are never useful (full/tests.rs:171-184)
    for _ in range(len(seen)):
        rp = orc.recode(np.stack(seen), k + L, k, rng.integers(0, 256, len(seen), dtype=np.uint8))
        assert S[dec.decode(rp)] == "PieceNotUseful"
    while not dec.is_already_decoded():
        dec.decode(orc.encode(src, rng.integers(0, 256, (1, k), dtype=np.uint8))[0])
    st, out = dec.get_decoded_data()
    assert st == 0 and np.array_equal(out, data)
