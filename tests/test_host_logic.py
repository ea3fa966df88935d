"""CPU: the product's host logic (librlnc_hip's decoder elimination core) against the oracle.

Checks, without a GPU, the deferred-transform decoder design (elimination.hpp): for every sequence of
decode() calls the product's accept/reject answers equal the reference algorithm's, and
T × (received data rows) equals the oracle's full-row RREF payload byte-for-byte.
"""
import numpy as np
import pytest

from oracle import np_oracle as npo
from oracle.oracle import OracleDecoder
from rlnc_amd.elimination import Elimination
from tests.conftest import hexarr

S = ["Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
     "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful", "ReceivedAllPieces",
     "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength", "InvalidOutputBuffer"]


def run_product(k, L, pieces, fixed):
    """Replays Decoder::decode on the product's elimination; returns statuses and T × D payload."""
    e = Elimination(k, len(pieces) if fixed else 0)
    store = {}
    sts = []
    for p in pieces:
        p = np.asarray(p, np.uint8)
        if e.rank == k:
            sts.append("ReceivedAllPieces")
            continue
        if p.size != k + L:
            sts.append("InvalidPieceLength")
            continue
        st, slot, keep = e.push(p[:k])
        sts.append(S[st])
        if keep:
            store[slot] = p[k:].copy()
    T = e.transform()
    D = np.zeros((T.shape[1], L), np.uint8)
    for s, row in store.items():
        D[s] = row
    payload = npo.matmul(T, D)[: e.rank]
    return sts, payload, e


@pytest.mark.parametrize("fixed", [False, True])
def test_golden_sequences(golden, fixed):
    for v in golden["decode"]:
        k, L = v["k"], v["L"]
        sts, payload, _ = run_product(k, L, [hexarr(p) for p in v["pieces"]], fixed)
        assert sts == v["statuses"], v["name"]
        assert payload.tobytes().hex() == v["payload"], v["name"]


def _random_sequence(rng, k, L, n, sparsity):
    pieces = []
    for _ in range(n):
        cv = rng.integers(0, 256, k, dtype=np.uint8)
        cv[rng.random(k) < sparsity] = 0
        pieces.append(np.concatenate([cv, rng.integers(0, 256, L, dtype=np.uint8)]))
    # duplicates and linear combinations of earlier pieces (dependent)
    for _ in range(n // 4):
        i, j = rng.integers(0, len(pieces), 2)
        c = int(rng.integers(1, 256))
        pieces.insert(int(rng.integers(0, len(pieces))), pieces[i] ^ npo.mul_table()[c][pieces[j]])
    return pieces


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("fixed", [False, True])
def test_random_sequences_match_oracle(seed, fixed):
    rng = np.random.default_rng(seed)
    k = int(rng.integers(1, 24))
    L = int(rng.integers(1, 40))
    sparsity = [0.0, 0.5, 0.8, 0.95][seed % 4]
    pieces = _random_sequence(rng, k, L, int(k * 1.5) + 2, sparsity)
    od = OracleDecoder(L, k)
    want = [S[od.decode(p)] for p in pieces]
    sts, payload, e = run_product(k, L, pieces, fixed)
    assert sts == want
    assert np.array_equal(payload, od.padded_payload())
    assert np.array_equal(e.coefficients(), od.matrix()[:, :k])


def test_slot_recycling_bounds_storage():
    # useless pieces must not grow the data store (recycled slots)
    rng = np.random.default_rng(3)
    k, L = 8, 4
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Elimination(k)
    coded = npo.encode(src, rng.integers(0, 256, (4, k), dtype=np.uint8))
    for p in coded:
        e.push(p[:k])
    for _ in range(50):  # recoded, all dependent
        r = npo.recode(coded, k, rng.integers(0, 256, 4, dtype=np.uint8))
        st, slot, keep = e.push(r[:k])
        assert S[st] == "PieceNotUseful" and not keep
    assert e.slots <= 2 * (k + 1)


def test_elimination_errors():
    from rlnc_amd.errors import RLNCError

    with pytest.raises(RLNCError) as ei:
        Elimination(0)
    assert ei.value == RLNCError.PieceCountZero


@pytest.mark.parametrize("k,sparsity,seed", [(64, 0.0, 1), (64, 0.9, 2), (130, 0.5, 3), (130, 0.97, 4),
                                             (200, 0.0, 5), (200, 0.98, 6)])
def test_large_k_sequences_match_oracle(k, sparsity, seed):
    """The row-by-row backward pass and the last-row forward pass (elimination.cpp) across the 64-column scan blocks:
    every status, the E rows' payload and the whole coefficient matrix equal the reference algorithm's."""
    rng = np.random.default_rng(seed)
    L = 6
    pieces = _random_sequence(rng, k, L, k + k // 2, sparsity)
    od = OracleDecoder(L, k)
    want = [S[od.decode(p)] for p in pieces]
    sts, payload, e = run_product(k, L, pieces, False)
    assert sts == want
    assert np.array_equal(payload, od.padded_payload())
    assert np.array_equal(e.coefficients(), od.matrix()[:, :k])
