"""GPU checks of the multi-GPU building blocks through the C ABI: bit realignment
(ndfl_bits_shift), range decode with a window (ndfl_inflate_range), deferred windows
(NDFL_DICT_DEFERRED + ndfl_inflate_resolve), and the whole sharded protocol with 2 ranks sharing
cuda:0 over gloo (host-staged exchanges)."""
import os
import random

import pytest

import oracle_lib as O
from corpus import mixed_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import ndfl
    ctx = ndfl.Context(0)
    # device tensors are written by torch kernels: run the codec on torch's stream (the context's
    # own stream is non-blocking and would not wait for them)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    return torch, ndfl, ctx


def test_bits_shift_matches_integer_shift(env):
    torch, ndfl, ctx = env
    rng = random.Random(5)
    for nbits in [1, 7, 8, 9, 31, 32, 33, 1000, 8 * 4096 + 3, 1 << 20]:
        nin = (nbits + 7) // 8
        src_b = bytes(rng.getrandbits(8) for _ in range(nin))
        v = int.from_bytes(src_b, "little") & ((1 << nbits) - 1)
        for off in (0, 1):                       # aligned and unaligned source
            src = torch.frombuffer(bytearray(b"\xAA" * off + src_b + b"\xFF" * 8), dtype=torch.uint8).cuda()
            for shift in range(8):
                nout = (nbits + shift + 7) // 8
                dst = torch.full((nout + 8,), 0x55, dtype=torch.uint8, device="cuda")
                ctx.bits_shift_raw(src.data_ptr() + off, nbits, shift, dst.data_ptr(), nout)
                got = bytes(dst[:nout].cpu().numpy())
                assert got == (v << shift).to_bytes(nout, "little"), (nbits, off, shift)
                assert bytes(dst[nout:].cpu().numpy()) == b"\x55" * 8


def _stream_and_seams(data, strategy="RLE_DYNAMIC", chunk=65536):
    comp = O.deflate(data, strategy, chunk)
    bits = O.block_bits(data, strategy, chunk)
    seams = [0]
    for b in bits:
        seams.append(seams[-1] + b)
    return comp, seams


@pytest.mark.parametrize("strategy", ["RLE_DYNAMIC", "FULL_DYNAMIC", "RLE_STATIC"])
def test_inflate_range_with_window_matches_oracle(env, strategy):
    torch, ndfl, ctx = env
    data = mixed_bytes(12 * 65536 + 999, seed=11)
    comp, seams = _stream_and_seams(data, strategy)
    dev_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    for a, b in [(0, 3), (3, 7), (5, 13), (12, 13), (1, 2)]:
        s_bit, e_bit = seams[a], seams[b] if b < len(seams) - 1 else None
        out_pre = a * 65536
        dict_len = min(32768, out_pre)
        window = data[out_pre - dict_len:out_pre]
        r0, ref, rbits = O.inflate_range(comp, s_bit, e_bit, window)
        assert r0 is None
        n = len(ref)
        out = torch.zeros(dict_len + n + 64, dtype=torch.uint8, device="cuda")
        if dict_len:
            out[:dict_len] = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda()
        r, olen, bits = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), s_bit, e_bit, out.data_ptr(), dict_len,
                                              n + 64, ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
        assert (r, olen, bits) == (0, n, rbits), (a, b)
        assert bytes(out[dict_len:dict_len + n].cpu().numpy()) == ref
        # host-memory variant (window staged by the library)
        hbuf = bytearray(window + bytes(n + 64))
        import ctypes
        cbuf = (ctypes.c_uint8 * len(hbuf)).from_buffer(hbuf)
        cin = ctypes.create_string_buffer(comp, len(comp))
        r, olen, bits = ctx.inflate_range_raw(ctypes.addressof(cin), len(comp), s_bit, e_bit, ctypes.addressof(cbuf),
                                              dict_len, n + 64, 0)
        assert (r, olen) == (0, n) and bytes(hbuf[dict_len:dict_len + n]) == ref


def test_inflate_range_dictionary_bound(env):
    torch, ndfl, ctx = env
    # a range whose first block copies from 1 byte back needs >= 1 byte of window
    data = b"\x07" * 200000
    comp, seams = _stream_and_seams(data)
    dev_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    out = torch.zeros(32768 + 200000, dtype=torch.uint8, device="cuda")
    r, olen, bits = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), seams[1], None, out.data_ptr(), 0, 200000,
                                          ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
    r0, _, _ = O.inflate_range(comp, seams[1], None, b"")
    assert r0 == "COPY_FROM_BEFORE_DICTIONARY_START"
    assert r == O.REASONS.index(r0) + 1
    out[:1] = 7
    r, olen, bits = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), seams[1], None, out.data_ptr(), 1, 200000,
                                          ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
    assert (r, olen) == (0, 200000 - 65536)


def test_range_end_must_be_block_boundary(env):
    torch, ndfl, ctx = env
    data = mixed_bytes(4 * 65536, seed=3)
    comp, seams = _stream_and_seams(data)
    dev_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    out = torch.zeros(4 * 65536 + 64, dtype=torch.uint8, device="cuda")
    r, _, _ = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), 0, seams[2] - 5, out.data_ptr(), 0, out.numel(),
                                    ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
    assert r == ndfl._lib.E_ARG


@pytest.mark.parametrize("seed", [1, 2])
def test_deferred_window_then_resolve(env, seed):
    torch, ndfl, ctx = env
    rng = random.Random(seed)
    # runs across every chunk seam + LZ77 (FULL) so chains read the window transitively
    parts = []
    for k in range(10):
        parts.append(mixed_bytes(50000, seed=seed * 100 + k))
        parts.append(bytes([rng.getrandbits(8)]) * rng.randint(20000, 90000))
    data = bytearray(b"".join(parts))
    data[4 * 65536 - 1000:4 * 65536 + 1000] = b"\x5a" * 2000    # the range starts inside a run
    data = bytes(data)
    for strategy in ("RLE_DYNAMIC", "FULL_DYNAMIC"):
        comp, seams = _stream_and_seams(data, strategy)
        dev_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
        a = 4
        pre = a * 65536
        window = data[pre - 32768:pre]
        r0, ref, _ = O.inflate_range(comp, seams[a], None, window)
        assert r0 is None
        out = torch.full((32768 + len(ref) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        r, olen, bits = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), seams[a], None, out.data_ptr(), 32768,
                                              len(ref) + 64, ndfl.IN_DEVICE | ndfl.OUT_DEVICE | ndfl.DICT_DEFERRED)
        assert (r, olen) == (0, len(ref))
        out[:32768] = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda()
        # the next rank's window first (ndfl_inflate_tail), then the resolve
        for n in (32768, 40000, 5):
            tail = torch.zeros(n, dtype=torch.uint8, device="cuda")
            assert ctx.inflate_tail_raw(n, tail.data_ptr())
            assert bytes(tail.cpu().numpy()) == (window + ref)[-n:]
        n_re = ctx.inflate_resolve()
        assert n_re >= 1
        assert bytes(out[32768:32768 + olen].cpu().numpy()) == ref
        with pytest.raises(ndfl.NdflError):
            ctx.inflate_resolve()                       # nothing pending any more


@pytest.mark.parametrize("seed,a,strategy", [(3, 4, "RLE_DYNAMIC"), (4, 4, "FULL_DYNAMIC"), (5, 1, "FULL_DYNAMIC")])
def test_tail_map_composes_to_tail_and_resolved_output(env, seed, a, strategy):
    """ndfl_inflate_tail_map on the real device decode: a deferred range decode's last n bytes as a
    map of its window, applied to the true window, equal ndfl_inflate_tail and the resolved output --
    for tails inside the range's output and tails longer than it (reaching into the window: the map
    then points those bytes back at their own window index), and a range whose output is shorter
    than the window (a = 1: a short first shard)."""
    torch, ndfl, ctx = env
    rng = random.Random(seed)
    parts = []
    for k in range(6):
        parts.append(mixed_bytes(30000, seed=seed * 10 + k))
        parts.append(bytes([rng.getrandbits(8)]) * rng.randint(100, 30000))
    data = (b"".join(parts) * 3)[:7 * 65536]
    chunk = 16384 if a == 1 else 65536
    comp, seams = _stream_and_seams(data, strategy, chunk)
    pre = a * chunk
    window = data[max(0, pre - 32768):pre]
    dict_len = len(window)
    # a range of one or two chunks: its output may be shorter than a window
    b = min(a + (1 if a == 1 else 2), len(seams) - 1)
    e_bit = seams[b] if b < len(seams) - 1 else None
    r0, ref, _ = O.inflate_range(comp, seams[a], e_bit, window)
    assert r0 is None
    dev_in = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    out = torch.full((dict_len + len(ref) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    r, olen, _ = ctx.inflate_range_raw(dev_in.data_ptr(), len(comp), seams[a], e_bit, out.data_ptr(), dict_len,
                                       len(ref) + 64, ndfl.IN_DEVICE | ndfl.OUT_DEVICE | ndfl.DICT_DEFERRED)
    assert (r, olen) == (0, len(ref))
    full = window + ref
    win_t = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda().long()
    for n in sorted({min(len(full), x) for x in (5, 4096, len(ref), len(ref) + 1000, 32768)}):
        m = torch.zeros(n, dtype=torch.int32, device="cuda")
        assert ctx.inflate_tail_map_raw(n, m.data_ptr())
        mm = m.long()
        lit = mm < 0
        assert bool((lit | ((mm >= 0) & (mm < dict_len))).all()), n
        got = torch.where(lit, mm & 0xFF, win_t[torch.where(lit, torch.zeros_like(mm), mm)] if dict_len else mm & 0xFF)
        assert bytes(got.to(torch.uint8).cpu().numpy()) == full[-n:], n
        # bytes the map takes from the window in the part before the range's output: themselves
        k0 = max(0, n - len(ref))
        if k0:
            idx = torch.arange(dict_len - k0, dict_len, device="cuda")
            assert bool((mm[:k0] == idx).all()), n
    out[:dict_len] = torch.frombuffer(bytearray(window), dtype=torch.uint8).cuda()
    for n in (min(len(full), 32768), 7):
        tail = torch.zeros(n, dtype=torch.uint8, device="cuda")
        assert ctx.inflate_tail_raw(n, tail.data_ptr())
        assert bytes(tail.cpu().numpy()) == full[-n:]
    ctx.inflate_resolve()
    assert bytes(out[dict_len:dict_len + olen].cpu().numpy()) == ref


def test_sharded_protocol_small_shards_one_gpu():
    """4 ranks on cuda:0 with 4 KiB shards: the encoder history and the decode window each span
    several earlier shards (composed through up to 3 tail maps whose tails reach into their own
    windows)."""
    from test_parallel_cpu import run_workers
    res = run_workers(4, dict(chunk_len=4096, chunks_per_rank=1, last_bytes=2000, seed=25,
                              strategy="FULL_DYNAMIC", seam_run=False, codec="device"))
    assert res[0]["stream_equal"] and all(r["gathered_equal"] for r in res)
    assert all(r["code"] == 0 and r["decoded_equal"] for r in res)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_protocol_ranks_one_gpu(world):
    """The whole sharded protocol with 2 and 3 ranks sharing cuda:0 over gloo; with 3, the middle
    rank passes its window on through ndfl_inflate_tail before its own resolve."""
    from test_parallel_cpu import run_workers
    res = run_workers(world, dict(chunk_len=65536, chunks_per_rank=6, last_bytes=300001, seed=9,
                                  strategy="RLE_DYNAMIC", seam_run=True, codec="device"))
    assert res[0]["stream_equal"]
    assert all(r["gathered_equal"] for r in res)      # the device gather onto rank 0
    assert all(r["code"] == 0 and r["decoded_equal"] for r in res)


def test_sharded_protocol_async_gather_into_reused_buffer():
    """bench.py's step shape on the GPU codec: the root gathers asynchronously into a preallocated
    buffer full of garbage while every rank decodes its shard; the gathered stream must equal the
    oracle's single-stream encoding."""
    from test_parallel_cpu import run_workers
    res = run_workers(3, dict(chunk_len=65536, chunks_per_rank=4, last_bytes=70001, seed=12,
                              strategy="RLE_DYNAMIC", seam_run=True, codec="device", async_gather=True))
    assert res[0]["stream_equal"] and all(r["gathered_equal"] for r in res)
    assert all(r["code"] == 0 and r["decoded_equal"] for r in res)


def test_sharded_protocol_window_chain_longer_than_tail_limit():
    """A middle rank whose whole output reads the window through dist-7 LZ77 chains far longer than
    ndfl_inflate_tail follows: the tail gives up (NDFL_E_UNSUPPORTED) and inflate_shard resolves
    first, then passes its last 32 KiB on; every rank's output and the gathered stream stay exact."""
    from test_parallel_cpu import run_workers
    res = run_workers(3, dict(chunk_len=65536, chunks_per_rank=6, last_bytes=100000, seed=13,
                              strategy="FULL_DYNAMIC", periodic=True, codec="device", count_tail_fallbacks=True))
    assert res[0]["stream_equal"] and all(r["gathered_equal"] for r in res)
    assert all(r["code"] == 0 and r["decoded_equal"] for r in res)
    assert res[1]["tail_fallbacks"] == 1, res


@pytest.mark.parametrize("stream", ["RLE_DYNAMIC", "zlib6", "FULL_DYNAMIC"])
def test_split_decode_of_foreign_stream_two_ranks_one_gpu(stream):
    """inflate_split on the GPU: a stream without a seam index (ours, Python zlib's, LZ77) decoded by
    2 ranks sharing cuda:0 over gloo from seams found by ndfl_inflate_sync; the joined output equals
    the data and both ranks took part."""
    from test_parallel_cpu import run_workers
    res = run_workers(2, dict(mode="split", n=2_000_000, seed=11, stream=stream, codec="device"))
    assert res[0]["equal"]
    assert all(r["code"] == 0 for r in res)
    assert res[0]["split"]


def test_inflate_sync_finds_true_boundaries(env):
    """ndfl_inflate_sync returns a real block boundary (one of the oracle's chunk seams) at or past
    the probe point, a few blocks on at most, for probes all over the stream."""
    torch, ndfl, ctx = env
    data = mixed_bytes(3_000_000, 21)
    comp = O.deflate(data)
    seams, acc = [], 0
    for v in O.block_bits(data):
        seams.append(acc)
        acc += v
    dev = torch.frombuffer(bytearray(comp + bytes(256)), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    for frac in (0.1, 0.33, 0.5, 0.77, 0.95):
        p = int(len(comp) * 8 * frac)
        s = ctx.inflate_sync_raw(dev.data_ptr(), len(comp), p, 8 << 20, ndfl.IN_DEVICE)
        assert s is not None and s >= p and s in seams, (frac, p, s)
        assert s < p + 3 * 65536 * 8            # within a few blocks
