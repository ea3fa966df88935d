"""Products on rows that are not 16-byte aligned -- the common case, since Encoder::new pads to
L = ceil((len + 1) / k) (encoder.rs:93-95) and a coded piece's data starts at byte k of its (k + L)-byte row.  On a
device whose queues execute 16-byte vector memory instructions at any byte address (probed when the first context is
created: rlnc_device_unaligned_vector_access) they take the vector kernels directly; elsewhere (or with
RLNC_ASSUME_ALIGNED_ONLY=1) kernels.hip's realigned path copies them through 16-byte scratch rows
(`realign_plan` / `realign_rows_kernel`).  Both paths checked bit for bit against the numpy checker and against the
same product on aligned copies, with the bytes around every misaligned output row (a coded piece's coefficient
header) left untouched; the realigned path in a child process with the variable set."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.gpu_util import dev, host, np_matmul

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    return rlnc_amd.Context(0)


def _desc(inp, in_off, in_row, coef, out, out_off, out_row, n_out, n_in, width, nobj, hdr=None, hdr_row=0):
    from rlnc_amd._lib import MatmulDesc

    return MatmulDesc(inp.data_ptr() + in_off, inp.stride(0), in_row, coef.data_ptr(), n_out * n_in, n_in,
                      out.data_ptr() + out_off, out.stride(0), out_row,
                      None if hdr is None else hdr.data_ptr(), 0 if hdr is None else hdr.stride(0), hdr_row,
                      n_out, n_in, width, nobj)


def _run(ctx, d):
    from rlnc_amd.errors import check

    check(ctx.lib.rlnc_gf256_matmul(ctx.h, C.byref(d)), ctx.lib)


# (n_out, n_in, width, nobj, input byte offset, input row pad, output byte offset, output row pad): every
# combination of misaligned base / row stride on either side, widths around the 4 KiB column block and its
# 16-byte slots, 1-3 output rows (the stream kernel) and 4+ (bit-sliced, 4- and 8-wave tiles)
CASES = [
    (64, 32, 4096, 2, 0, 5, 0, 0),           # input rows at an odd stride
    (64, 32, 4096, 2, 0, 0, 3, 1),           # output only
    (32, 30, 8192 + 7, 3, 30, 1, 30, 1),      # coded-piece framing: data at byte k of (k + L)-byte rows
    (16, 16, 12288 + 3, 2, 1, 3, 2, 7),
    (1, 33, 4096 * 3 + 1, 2, 33, 0, 33, 0),   # one coded piece (stream kernel), header before it
    (3, 7, 5000, 1, 7, 2, 5, 2),
    (100, 17, 4096 * 2 + 9, 1, 17, 4, 100, 4),
    (8, 8, 4096, 4, 8, 0, 8, 0),
    (40, 1, 4096 + 15, 2, 1, 1, 2, 2),
]


@pytest.mark.parametrize("n_out,n_in,W,nobj,ioff,ipad,ooff,opad", CASES)
def test_realigned_matmul(ctx, n_out, n_in, W, nobj, ioff, ipad, ooff, opad):
    import torch

    rng = np.random.default_rng(n_out * 31 + n_in * 7 + W + nobj + ioff + ooff)
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    coef[:, 0, :] = 1
    data = rng.integers(0, 256, (nobj, n_in, W), dtype=np.uint8)
    in_row = W + ipad + ioff
    inbuf = np.zeros((nobj, n_in * in_row + 64), np.uint8)
    for o in range(nobj):
        for j in range(n_in):
            inbuf[o, ioff + j * in_row: ioff + j * in_row + W] = data[o, j]
    out_row = W + opad + ooff
    sentinel = rng.integers(0, 256, (nobj, n_out * out_row + 64), dtype=np.uint8)
    inp, cf, out = dev(inbuf), dev(coef), dev(sentinel)
    _run(ctx, _desc(inp, ioff, in_row, cf, out, ooff, out_row, n_out, n_in, W, nobj))
    got = host(out)
    for o in range(nobj):
        want = np_matmul(coef[o], data[o])
        exp = sentinel[o].copy()
        for i in range(n_out):
            exp[ooff + i * out_row: ooff + i * out_row + W] = want[i]
        assert np.array_equal(got[o], exp), o  # every product byte, and nothing outside the rows written
    torch.cuda.synchronize()


def test_realigned_headers(ctx):
    """encode_batch framing through a misaligned view: coefficient header + data in (k + L)-byte rows, L odd."""
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(77)
    nobj, k, L, n = 3, 30, 4096 * 2 + 11, 45
    src = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
    coeffs = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    out = torch.empty((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(dev(src), dev(coeffs), out, ctx)
    got = host(out)
    for o in range(nobj):
        assert np.array_equal(got[o, :, :k], coeffs[o])
        assert np.array_equal(got[o, :, k:], np_matmul(coeffs[o], src[o])), o


def test_realigned_chunks_match_aligned(ctx):
    """Beyond the 512 MiB realignment budget the product runs in column chunks (and object chunks): the result equals
    the same product on aligned copies, byte for byte."""
    import torch

    nobj, n_out, n_in, W = 3, 64, 64, (1 << 21) + 5
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    in_row = W + 3
    inbuf = torch.randint(0, 256, (nobj, n_in * in_row + 16), dtype=torch.uint8, device="cuda:0", generator=g)
    coef = torch.randint(0, 256, (nobj, n_out, n_in), dtype=torch.uint8, device="cuda:0", generator=g)
    out_row = W + 1
    outbuf = torch.zeros((nobj, n_out * out_row + 16), dtype=torch.uint8, device="cuda:0")
    _run(ctx, _desc(inbuf, 3, in_row, coef, outbuf, 7, out_row, n_out, n_in, W, nobj))
    Wa = (W + 15) // 16 * 16
    src_al = torch.zeros((nobj, n_in, Wa), dtype=torch.uint8, device="cuda:0")
    src_al[:, :, :W] = inbuf[:, 3:3 + n_in * in_row].reshape(nobj, n_in, in_row)[:, :, :W]
    out_al = torch.zeros((nobj, n_out, Wa), dtype=torch.uint8, device="cuda:0")
    _run(ctx, _desc(src_al, 0, Wa, coef, out_al, 0, Wa, n_out, n_in, W, nobj))
    got = outbuf[:, 7:7 + n_out * out_row].reshape(nobj, n_out, out_row)[:, :, :W]
    assert torch.equal(got, out_al[:, :, :W])
    assert int(outbuf[:, :7].count_nonzero()) == 0 and int(outbuf[:, 7 + n_out * out_row:].count_nonzero()) == 0
    # the pad byte after every row (out_row = W + 1) untouched
    assert int(outbuf[:, 7:7 + n_out * out_row].reshape(nobj, n_out, out_row)[:, :, W:].count_nonzero()) == 0
    # spot-check one object's rows against the numpy checker on a slice of columns
    cols = slice(W - 4099, W)
    want = np_matmul(host(coef[1]), host(src_al[1, :, cols]))
    assert np.array_equal(host(got[1, :, cols]), want)


def test_unaligned_probe_reports(ctx):
    v = ctx.lib.rlnc_device_unaligned_vector_access(0)
    assert v in (0, 1), v
    assert ctx.lib.rlnc_device_unaligned_vector_access(63) == -1  # no context there: not probed


def _forced_main():
    """Child process (RLNC_ASSUME_ALIGNED_ONLY=1): every CASES product and the header framing on the realigned path."""
    import rlnc_amd

    c = rlnc_amd.Context(0)
    assert c.lib.rlnc_device_unaligned_vector_access(0) == 0
    for case in CASES:
        test_realigned_matmul(c, *case)
    test_realigned_headers(c)
    test_realigned_chunks_match_aligned(c)
    print("forced realigned path ok")


def test_realigned_path_forced():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RLNC_ASSUME_ALIGNED_ONLY="1", PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--forced"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "forced realigned path ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


if __name__ == "__main__" and "--forced" in sys.argv:
    _forced_main()
