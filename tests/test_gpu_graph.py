"""GPU: the batch API under HIP-graph capture (bench.py --graph), including a capture that is the process's first
use of the shared-set kernel (its one-time table-address probe cannot run inside a capture: that launch takes the
bit-identical variant-6 program).  Runs in a child process so that the capture really is the first use.  Context
workspaces must have grown before a capture (an eager call of the same shape), like torch's own warm-up rule."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, ROOT)
import numpy as np
import torch
import rlnc_amd
from rlnc_amd import batch

ctx = rlnc_amd.Context(0)
rng = np.random.default_rng(5)
B, k, L, n = 3, 32, 3 * 4096 + 32, 40
src = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
co = torch.from_numpy(rng.integers(0, 256, (B, n, k), dtype=np.uint8)).cuda()
cap = torch.zeros((B, n, k + L), dtype=torch.uint8, device="cuda")
# workspaces grow outside a capture (as torch's own warm-up rule): one eager call with variant 6, so that the
# captured shared-set call below (variant 7, or 8 with its 64-row tiles) is the first use of the shared-set kernel
# (its address probe is not yet done); 40 rows take as much scratch in 32- as in 64-row tiles
ctx.set_kernel_variant(6)
batch.encode_batch(src, co, cap, ctx)
torch.cuda.synchronize()
ctx.set_kernel_variant(VARIANT)
cap.zero_()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        batch.encode_batch(src, co, cap, ctx)
g.replay()
torch.cuda.synchronize()
eager = torch.zeros_like(cap)
batch.encode_batch(src, co, eager, ctx)
torch.cuda.synchronize()
assert torch.equal(cap, eager), "captured encode differs from eager"
cap.zero_()
g.replay()
torch.cuda.synchronize()
assert torch.equal(cap, eager), "replay differs"
# the captured graph holds the context's workspace addresses: a larger eager call on the same context must
# refuse to grow them (instead of freeing memory the graph still writes), and the graph stays correct
big_src = torch.from_numpy(rng.integers(0, 256, (4 * B, k, L), dtype=np.uint8)).cuda()
big_co = torch.from_numpy(rng.integers(0, 256, (4 * B, n, k), dtype=np.uint8)).cuda()
big = torch.zeros((4 * B, n, k + L), dtype=torch.uint8, device="cuda")
try:
    batch.encode_batch(big_src, big_co, big, ctx)
    raise SystemExit("a workspace grew after a capture")
except rlnc_amd.RLNCError as e:
    assert e == rlnc_amd.RLNCError.InvalidArgument, e
cap.zero_()
g.replay()
torch.cuda.synchronize()
assert torch.equal(cap, eager), "replay after the refused call differs"
ctx2 = rlnc_amd.Context(0)  # another context serves the larger shape
batch.encode_batch(big_src, big_co, big, ctx2)
ref = torch.zeros_like(big)
ctx2.set_kernel_variant(0)
batch.encode_batch(big_src, big_co, ref, ctx2)
torch.cuda.synchronize()
assert torch.equal(big, ref)
print("graph ok")
"""


@pytest.mark.parametrize("variant", [7, 8])
def test_encode_batch_under_graph_capture_first_use(variant):
    code = CHILD.replace("ROOT", repr(ROOT)).replace("VARIANT", str(variant))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "graph ok" in r.stdout


# Descriptor tables under capture (wire.hip upload_table): a captured pad call and a captured ragged decode keep
# their own tables, so eager calls with OTHER descriptors between the capture and a replay cannot change what the
# replay reads (the captured tables are written by kernels that carry the bytes, into a region never reused).
CHILD_TABLES = r"""
import sys
sys.path.insert(0, ROOT)
import ctypes as C
import numpy as np
import torch
import rlnc_amd
from rlnc_amd import _lib, batch
from oracle.oracle import Oracle

orc = Oracle()
ctx = rlnc_amd.Context(0)
rng = np.random.default_rng(11)
shapes = [(1000, 3), (5000, 16), (4096 * 2 - 1, 2)]


def pad_set():
    datas = [torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).cuda() for n, _ in shapes]
    outs = [torch.zeros(k * orc.piece_byte_len(n, k), dtype=torch.uint8, device="cuda") for n, k in shapes]
    arr = (_lib.PadDesc * len(shapes))(*[_lib.PadDesc(d.data_ptr(), n, k, o.data_ptr(), 0)
                                         for (n, k), d, o in zip(shapes, datas, outs)])
    return datas, outs, arr


def decode_set(B=6):
    objs, srcs = [], []
    for o in range(B):
        k, L = (16, 4096) if o % 2 else (40, 3 * 4096 + 16)
        src = orc.pad(rng.integers(0, 256, k * L - 3, dtype=np.uint8), k)
        pc = torch.from_numpy(orc.encode(src, rng.integers(0, 256, (k + 2, k), dtype=np.uint8))).cuda()
        objs.append((pc, k, torch.zeros((k, L), dtype=torch.uint8, device="cuda")))
        srcs.append(src)
    return objs, srcs


def pad(arr):
    ctx.use_torch_stream()
    assert ctx.lib.rlnc_pad_batch_device(ctx.h, arr, len(shapes)) == 0


X = pad_set()
A = decode_set()
if WARM_PAD:
    pad(X[2])  # eager warm-up: workspaces, the capture arena, the block-table probe
batch.decode_ragged(A[0], ctx)
torch.cuda.synchronize()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        pad(X[2])
        res = batch.decode_ragged(A[0], ctx)
torch.cuda.synchronize()
Y = pad_set()  # other descriptors, same sizes, eager, between the capture and the replay
B_ = decode_set()
pad(Y[2])
resB = batch.decode_ragged(B_[0], ctx)
torch.cuda.synchronize()
for _ in range(EXTRA_DECODES):  # more eager calls: the staging ring rotates onto slots the warm-up never grew
    C_ = decode_set()
    batch.decode_ragged(C_[0], ctx)
    torch.cuda.synchronize()
    for (pc, k, dec), src in zip(C_[0], C_[1]):
        assert np.array_equal(dec.cpu().numpy(), src), "extra eager ragged decode"
for (n, k), d, o in zip(shapes, Y[0], Y[1]):
    assert np.array_equal(o.cpu().numpy(), orc.pad(d.cpu().numpy(), k).reshape(-1)), "eager pad"
for (pc, k, dec), src in zip(B_[0], B_[1]):
    assert np.array_equal(dec.cpu().numpy(), src), "eager ragged decode"
for o in X[1]:
    o.zero_()
for _, _, dec in A[0]:
    dec.zero_()
res[1].fill_(-1)
g.replay()
torch.cuda.synchronize()
for (n, k), d, o in zip(shapes, X[0], X[1]):
    assert np.array_equal(o.cpu().numpy(), orc.pad(d.cpu().numpy(), k).reshape(-1)), "replayed pad"
for (pc, k, dec), src in zip(A[0], A[1]):
    assert np.array_equal(dec.cpu().numpy(), src), "replayed ragged decode"
assert (res[1].cpu().numpy() == 0).all(), "replayed statuses"
print("tables ok")
"""


@pytest.mark.parametrize("warm_pad,extra", [(True, 0), (False, 2)], ids=["pad+decode-warmup", "decode-warmup+2-eager"])
def test_descriptor_tables_survive_other_eager_calls_before_replay(warm_pad, extra):
    """The capture's tables live in the capture arena; eager calls after the capture stage through the pinned ring,
    whose slots grow on their own first use even on a graph-bound context (with the warm-up a single
    ragged decode, later eager decodes land on ring slots that were never grown)."""
    code = CHILD_TABLES.replace("ROOT", repr(ROOT)).replace("WARM_PAD", repr(warm_pad)).replace(
        "EXTRA_DECODES", str(extra))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tables ok" in r.stdout


def test_small_object_decode_under_graph_capture():
    """configs[0]'s decode form under capture: the small-object elimination answering the marker scan from the
    payload tail (RrefParams::tail_status) and the product's workgroups scanning the all-zero tails
    (MatmulParams::scan_need) -- captured after an eager warm-up, replayed into zeroed outputs, equal to the eager
    decode, which is checked against the source."""
    import numpy as np
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    rng = np.random.default_rng(9)
    B, k, L = 2048, 16, 4096
    src = rng.integers(0, 256, (B, k * L), dtype=np.uint8)
    src[0::3, -1] = 0x81  # marker last: decided by the tail
    src[1::3, 200:] = 0   # marker early, a long zero tail: scanned by the product's workgroup
    src[1::3, 199] = 0x81
    src_d = torch.from_numpy(src.reshape(B, k, L)).cuda()
    co = torch.from_numpy(rng.integers(0, 256, (B, k, k), dtype=np.uint8)).cuda()
    pieces = torch.empty((B, k, k + L), dtype=torch.uint8, device="cuda")
    batch.encode_batch(src_d, co, pieces, ctx)

    def outputs():
        return (torch.zeros((B, k, L), dtype=torch.uint8, device="cuda"),
                torch.full((B, k), -1, dtype=torch.int32, device="cuda"),
                torch.full((B,), -1, dtype=torch.int32, device="cuda"),
                torch.full((B,), -1, dtype=torch.int64, device="cuda"))

    eager = outputs()
    batch.decode_batch_device(pieces, k, *eager, ctx)  # also the warm-up: workspaces grow here
    torch.cuda.synchronize()
    cap = outputs()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            batch.decode_batch_device(pieces, k, *cap, ctx)
    for t in cap:
        t.fill_(0)
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(cap, eager):
        assert torch.equal(a, b)
    ost, dl = eager[2].cpu().numpy(), eager[3].cpu().numpy()
    full = (eager[1] == 0).sum(1).cpu().numpy() == k
    dec = eager[0].cpu().numpy().reshape(B, k * L)
    assert full.sum() > B * 0.9
    for o in np.nonzero(full)[0]:
        assert np.array_equal(dec[o], src[o]), o
        if o % 3 == 0:
            assert ost[o] == 0 and dl[o] == k * L - 1, o
        elif o % 3 == 1:
            assert ost[o] == 0 and dl[o] == 199, o


# stream-context eviction must skip a context whose stream is mid-capture even when the capture is on a
# stream that is not torch's current one.  The capture status is asked through librlnc_hip (rlnc_stream_is_capturing,
# the runtime torch shares), and an error counts as capturing.
CHILD_EVICT = r"""
import sys
sys.path.insert(0, ROOT)
import numpy as np
import torch
import rlnc_amd
from rlnc_amd import batch, context

rng = np.random.default_rng(21)
B, k, L, n = 2, 8, 4096, 6
src = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
co = torch.from_numpy(rng.integers(0, 256, (B, n, k), dtype=np.uint8)).cuda()
ref = torch.zeros((B, n, k + L), dtype=torch.uint8, device="cuda")
batch.encode_batch(src, co, ref, rlnc_amd.Context(0))
torch.cuda.synchronize()
cap_s = torch.cuda.Stream()
others = [torch.cuda.Stream() for _ in range(context.STREAM_CONTEXTS_PER_THREAD + 2)]
# the capture stream's context first (least recently used), then enough others to fill the per-thread cap
for s in [cap_s] + others[:context.STREAM_CONTEXTS_PER_THREAD - 1]:
    with torch.cuda.stream(s):
        out = torch.zeros_like(ref)
        batch.encode_batch(src, co, out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
key = (0, cap_s.cuda_stream)
assert key in context._tls.sctxs
assert not context._stream_capturing(cap_s.cuda_stream)
x = torch.zeros(16, device="cuda")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=cap_s, capture_error_mode="relaxed"):
    x.add_(1)  # torch work captured on cap_s; no rlnc call on cap_s, so its context is not graph-bound
    assert context._stream_capturing(cap_s.cuda_stream)
    assert torch.cuda.current_stream().cuda_stream == cap_s.cuda_stream
    # eager rlnc calls on fresh streams (not the current, capturing one): each new stream context overflows the
    # cap; eviction must pass over cap_s's context (closing it would synchronise a capturing stream)
    outs = []
    for s in others[context.STREAM_CONTEXTS_PER_THREAD - 1:]:
        with torch.cuda.stream(s):
            outs.append(torch.zeros_like(ref))
            batch.encode_batch(src, co, outs[-1])
        s.synchronize()
    assert key in context._tls.sctxs, "the capturing stream's context was evicted"
    x.add_(1)
for out in outs:  # compared outside the capture (a comparison on the capturing stream would synchronise it)
    assert torch.equal(out, ref)
g.replay()
torch.cuda.synchronize()
assert torch.equal(x, torch.full_like(x, 2)), x
assert not context._stream_capturing(cap_s.cuda_stream)
# outside the capture the next overflow may evict it again
with torch.cuda.stream(others[0]):
    out = torch.zeros_like(ref)
    batch.encode_batch(src, co, out)
torch.cuda.synchronize()
assert torch.equal(out, ref)
assert len(context._tls.sctxs) <= context.STREAM_CONTEXTS_PER_THREAD
print("evict ok")
"""


def test_stream_context_eviction_skips_capturing_non_current_stream():
    code = CHILD_EVICT.replace("ROOT", repr(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "evict ok" in r.stdout
