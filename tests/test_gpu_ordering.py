"""Stream ordering at the C ABI (include/ndfl.h, ndfl_ctx_set_stream): device buffers handed to the
library right after an asynchronous torch producer -- no host synchronize in between -- must be
read and written in order with that producer, and the results must equal the oracle's.

The round-2 config-3 fault came from exactly this: the context's own non-blocking stream ran the
library's staging copy while torch's corpus kernels were still writing the input.  Each test here
queues a long chain of torch kernels and calls the library immediately:
  * on torch's default stream (the C ABI's default rule: ordered after the NULL stream);
  * on a side stream made current with torch.cuda.stream (the Python Context binds it);
  * with an output block the caching allocator hands out again while queued kernels still write it;
  * for the decoder, an input stream still being copied into place.
Reference semantics: bit-exact output, D/comp/Lz77Huffman.java:62-130, D/decomp/Open.java:83-124.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

N = 24 << 20          # bytes: big enough that the producer chain runs for milliseconds


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as M
    return M


def _slow_corpus(torch, n, seed, rounds=40):
    """Runs of small bytes and noise, produced by `rounds` dependent kernels on the current stream."""
    x = torch.arange(n, device="cuda", dtype=torch.int64) * (seed | 1)
    for _ in range(rounds):
        x = (x * 6364136223846793005 + 1442695040888963407) & 0x7FFFFFFFFFFFFFFF
    r = (x >> 40) & 255
    runs = (torch.arange(n, device="cuda", dtype=torch.int64) >> 7) & 3
    return torch.where(r < 96, runs, r).to(torch.uint8)


def _deflate_dev(ndfl, ctx, torch, data, out=None):
    L = ndfl._lib.load()
    n = data.numel()
    cap = L.ndfl_deflate_bound(n, 65536) + 64
    if out is None:
        out = torch.empty(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, 3, True, 0, out.data_ptr(), cap,
                                   ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
    return out, eb


def test_deflate_right_after_producer_default_stream(ndfl):
    import torch
    ctx = ndfl.Context(0)                      # no set_stream: the default ordering rule
    for seed in (1, 2, 3):
        data = _slow_corpus(torch, N, seed)
        out, eb = _deflate_dev(ndfl, ctx, torch, data)      # no synchronize before this call
        host = data.cpu().numpy().tobytes()
        exp = O.deflate(host)
        assert (eb + 7) // 8 == len(exp)
        assert bytes(out[:len(exp)].cpu().numpy()) == exp


def test_deflate_right_after_producer_side_stream(ndfl):
    import torch
    ctx = ndfl.Context(0)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        data = _slow_corpus(torch, N, 7)
        out, eb = _deflate_dev(ndfl, ctx, torch, data)
    side.synchronize()
    exp = O.deflate(data.cpu().numpy().tobytes())
    assert (eb + 7) // 8 == len(exp) and bytes(out[:len(exp)].cpu().numpy()) == exp


def test_output_block_reused_by_the_allocator(ndfl):
    """A block freed while queued torch kernels still write it, handed out again as the output."""
    import torch
    ctx = ndfl.Context(0)
    L = ndfl._lib.load()
    data = _slow_corpus(torch, N, 11, rounds=2)
    exp = O.deflate(data.cpu().numpy().tobytes())
    cap = L.ndfl_deflate_bound(N, 65536) + 64
    for _ in range(3):
        scratch = torch.zeros(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
        for _ in range(60):
            scratch.add_(1)                    # queued writers of the block
        ptr = scratch.data_ptr()
        del scratch
        out = torch.empty(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
        reused = out.data_ptr() == ptr
        out, eb = _deflate_dev(ndfl, ctx, torch, data, out)
        assert (eb + 7) // 8 == len(exp)
        assert bytes(out[:len(exp)].cpu().numpy()) == exp, f"output corrupted (block reused: {reused})"


def test_inflate_right_after_producer(ndfl):
    import torch
    ctx = ndfl.Context(0)
    rng = np.random.default_rng(5)
    host = np.repeat(rng.integers(0, 5, N // 64, dtype=np.uint8), 64).tobytes()
    comp = O.deflate(host)
    src = torch.from_numpy(np.frombuffer(comp, dtype=np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    for _ in range(3):
        dev = torch.zeros(len(comp) + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
        junk = torch.zeros_like(dev)
        for _ in range(40):
            junk.add_(3)                       # keep the stream busy before the copy lands
        dev[:len(comp)].copy_(src)
        out = torch.empty(N + 64, dtype=torch.uint8, device="cuda")
        r, olen, bits = ctx.inflate_raw(dev.data_ptr(), len(comp), out.data_ptr(), out.numel(),
                                        ndfl.IN_DEVICE | ndfl.OUT_DEVICE | ndfl.IN_PADDED)
        assert r == 0 and olen == N and (bits + 7) // 8 == len(comp)
        assert bytes(out[:N].cpu().numpy()) == host
