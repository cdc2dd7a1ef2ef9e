"""GPU parity at the BASELINE.json configurations' own shapes, through the C ABI:

  * config 2: the 64 MiB .gz of stored + fixed-Huffman blocks (tests/corpus.py c2_gzip, PCG64 seed
    0xC2), decoded through GzipInputStream and compared byte for byte with the oracle's gunzip;
  * config 5: the random+repeat corpus (corpus.c5_random_repeat, seed 0xC5): a 256 MiB RLE_DYNAMIC
    GPU encode equal to the oracle's bytes, and the GPU round trip;
  * streams with more dynamic headers per 64 KiB finder segment than the finder keeps (SEG_CAP = 256,
    inflate_kernels.hip): chunk_len = 64 RLE_DYNAMIC, decoded equal to the oracle;
  * the one-kernel encoder (NDFL_DEFLATE_FUSED=1) against the oracle.
"""
import io
import os

import numpy as np
import pytest

import corpus
import knobs
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as N
    return N


@pytest.fixture(scope="module")
def ctx(ndfl):
    import torch
    c = ndfl.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)     # ordered with torch's kernels
    return c


def test_config2_gzip_64MiB(ndfl, ctx):
    gz, raw, data = corpus.c2_gzip(64 << 20)
    assert len(raw) >= 64 << 20
    reason, out, hdr, end = O.gunzip(gz)
    assert reason is None and out == data and end == len(gz)
    g = ndfl.GzipInputStream(io.BytesIO(gz), context=ctx)
    got = g.readall()
    assert got == out
    assert g.getMetadata().operatingSystem == "UNIX"
    # the raw stream alone: output, exact end bit
    r, o2, bits = ctx.inflate(raw)
    assert r is None and o2 == data and (bits + 7) // 8 == len(raw)


def test_config5_random_repeat_256MiB(ndfl, ctx):
    import torch
    a = corpus.c5_random_repeat(256 << 20)
    host = a.tobytes()
    exp = O.deflate(host)
    dev = torch.from_numpy(a).cuda()
    L = ndfl._lib.load()
    n = dev.numel()
    cap = L.ndfl_deflate_bound(n, 65536) + 64
    comp = torch.empty(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
    eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, dev.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, D)
    cb = (eb + 7) // 8
    assert cb == len(exp)
    assert bytes(comp[:cb].cpu().numpy()) == exp
    comp[cb:cb + ndfl.IN_PAD_BYTES].zero_()
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r, olen, bits = ctx.inflate_raw(comp.data_ptr(), cb, dec.data_ptr(), dec.numel(), D | ndfl.IN_PADDED)
    assert r == 0 and olen == n and bits == eb
    assert torch.equal(dec[:n], dev)


@pytest.mark.parametrize("chunk_len", [64, 200])
def test_more_headers_than_segment_cap(ctx, chunk_len):
    """~700 dynamic headers per 64 KiB of stream at chunk_len 64: the finder keeps 256 per segment,
    the rest are reached by chain continuation; output must still equal the oracle's."""
    rng = np.random.default_rng(chunk_len)
    parts = []
    for _ in range(3000):
        if rng.random() < 0.5:
            parts.append(bytes([int(rng.integers(0, 4))]) * int(rng.integers(1, 300)))
        else:
            parts.append(rng.integers(0, 16, int(rng.integers(1, 200)), dtype=np.uint8).tobytes())
    data = b"".join(parts)[:300_000]
    comp = O.deflate(data, "RLE_DYNAMIC", chunk_len=chunk_len)
    assert ctx.deflate(data, "RLE_DYNAMIC", chunk_len=chunk_len) == comp
    r, out, bits = ctx.inflate(comp)
    oreason, oout, obits = O.inflate(comp)
    assert r is None and oreason is None and out == oout == data and bits == obits


def test_fused_encoder_matches_oracle(ctx):
    rng = np.random.default_rng(5)
    datas = [b"", b"\x00" * 70000, rng.integers(0, 256, 200_003, dtype=np.uint8).tobytes(),
             corpus.c4_mixed(3 << 20).numpy().tobytes()]
    fctx = knobs.context(NDFL_DEFLATE_FUSED=1)
    for d in datas:
        for strategy in ["RLE_DYNAMIC", "LITERAL_STATIC"]:
            assert fctx.deflate(d, strategy) == O.deflate(d, strategy), (len(d), strategy)
