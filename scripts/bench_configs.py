"""Measure the other BASELINE.json configurations on one MI355X (bench.py reports config 4).

    c1  gzip of 1 MiB of zeros through the stream API (host buffers; plumbing)
    c2  decompress a 64 MiB .gz of stored + fixed-Huffman (LZ77, dist 1..32768) blocks
        (tests/corpus.py c2_gzip; device-resident input -> output)
    c3  FULL_DYNAMIC (LZ77 + dynamic Huffman) compress of 1 GiB enwik-style text, device-resident;
        the WHOLE stream checked against the oracle (chunk-parallel on 16 host threads: a
        FULL_DYNAMIC block depends only on its chunk and 32 KiB of raw history,
        D/comp/Lz77Huffman.java:71-84), so the ratio is the reference's
    c5  the 16 GiB random+repeat round trip on one GPU (RLE_DYNAMIC; corpus.c5_device), device-resident,
        the whole stream checked against the oracle

Each config prints one JSON line; the oracle (1 thread) is timed on a bounded sample beside it.
Run on the GPU box: python scripts/bench_configs.py [c1 c2 c3 c5].
"""
import ctypes
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ndfl  # noqa: E402
import corpus  # noqa: E402
import oracle_lib as O  # noqa: E402

MIB = 1 << 20
DEV = ndfl.IN_DEVICE | ndfl.OUT_DEVICE


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def c1(ctx):
    data = b"\x00" * MIB
    meta = ndfl.GzipMetadata("DEFLATE", False, 1_700_000_000, 0, "UNIX", None, "zeros_1MiB.bin", None, True)

    def run():
        b = io.BytesIO()
        g = ndfl.GzipOutputStream(b, meta, context=ctx)
        g.write(data)
        g.finish()
        return b.getvalue()
    out = run()
    exp = O.gzip_compress(data, name=b"zeros_1MiB.bin", mtime=1_700_000_000, os_=3, header_crc=True)
    dt = timed(run, 20)
    t = time.perf_counter()
    for _ in range(5):
        O.gzip_compress(data, name=b"zeros_1MiB.bin", mtime=1_700_000_000, os_=3, header_crc=True)
    tc = (time.perf_counter() - t) / 5
    return {"config": "c1: gzip 1 MiB zeros (stream API, host buffers)", "bit_exact": out == exp,
            "gz_bytes": len(out), "input_MiBps": round(1 / dt, 1), "ms": round(dt * 1e3, 3),
            "cpu_oracle_MiBps": round(1 / tc, 1)}


def c2(ctx):
    # the -m gpu test's corpus (tests/corpus.py c2_gzip: stored + zlib Z_FIXED blocks, seed 0xC2)
    t = time.perf_counter()
    gz, raw, data = corpus.c2_gzip(64 * MIB)
    gen_s = time.perf_counter() - t
    comp_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    out = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    res = {}

    def run():
        r, olen, bits = ctx.inflate_raw(comp_dev.data_ptr(), len(raw), out.data_ptr(), out.numel(), DEV)
        res.update(r=r, olen=olen)
        res["crc"] = ctx.crc32(out[:olen], flags=ndfl.IN_DEVICE)
    dt = timed(run, 5)
    ok = res["r"] == 0 and res["olen"] == len(data) and bytes(out[:len(data)].cpu().numpy()) == data \
        and res["crc"] == O.crc32(data)
    # CPU: oracle gunzip of the same file, 16 MiB-of-output sample
    t = time.perf_counter()
    reason = O.gunzip(gz)[0]
    tc = time.perf_counter() - t
    return {"config": "c2: decompress 64 MiB .gz of stored + fixed-Huffman blocks (device-resident)", "bit_exact": ok,
            "gz_bytes": len(gz), "out_bytes": len(data), "input_MiBps": round(len(raw) / dt / MIB, 1),
            "output_MiBps": round(len(data) / dt / MIB, 1), "ms": round(dt * 1e3, 3),
            "timings": ctx.timings(), "cpu_oracle_input_MiBps": round(len(gz) / tc / MIB, 1),
            "cpu_oracle_ok": reason is None, "fixture_gen_s": round(gen_s, 1)}


def c3(ctx):
    n = 1 << 30
    data = corpus.c3_text(n, device="cuda")
    cap = ndfl._lib.load().ndfl_deflate_bound(n, 65536) + 64
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    st = {}

    def run():
        eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, ndfl.Lz77Huffman.FULL_DYNAMIC, True,
                                       0, out.data_ptr(), cap, DEV)
        st["eb"] = eb
        st["td"] = ctx.timings()["deflate"]
    dt = timed(run, 2)
    comp = (st["eb"] + 7) // 8
    from bench import verify_stream
    v = verify_stream(data, None, True, out, st["eb"], 16, strategy="FULL_DYNAMIC")
    pre = 16 * MIB
    host = data[:pre].cpu().numpy().tobytes()
    t = time.perf_counter()
    O.deflate(host, "FULL_DYNAMIC")
    tc = time.perf_counter() - t
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    r, olen, _ = ctx.inflate_raw(out.data_ptr(), comp, dec.data_ptr(), dec.numel(), DEV)
    rt = r == 0 and olen == n and torch.equal(dec[:n], data)
    return {"config": "c3: FULL_DYNAMIC compress 1 GiB text (LZ77 + dynamic Huffman, device-resident)",
            "input_MiBps": round(n / dt / MIB, 1), "ms": round(dt * 1e3, 1), "ratio": round(comp / n, 4),
            "bit_exact": v["bit_exact"], "verify": v, "round_trip_ok": rt,
            "deflate_device_ms": round(st["td"], 2), "cpu_oracle_MiBps": round(pre / tc / MIB, 2),
            "cpu_oracle_sample": "first 16 MiB, 1 thread"}


def c5(ctx, n=16 << 30):
    """Config 5 as BASELINE.json defines it: a 16 GiB random+repeat stream (corpus.c5_device, seed
    0xC5, generated on the device, not tiled), RLE_DYNAMIC compress then inflate on one GPU
    (288 GB HBM holds input, stream, output and the decoder's scratch).  bit_exact: the whole
    stream against the oracle (chunk-parallel on 16 host threads, bench.verify_stream)."""
    from bench import verify_stream
    t0 = time.perf_counter()
    data = corpus.c5_device(n, device="cuda")
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    cap = ndfl._lib.load().ndfl_deflate_bound(n, 65536) + 64
    comp = torch.empty(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    st = {}

    def run():
        t = time.perf_counter()
        eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, DEV)
        t1 = time.perf_counter()
        st["td"] = ctx.timings()["deflate"]
        cb = (eb + 7) // 8
        comp[cb:cb + ndfl.IN_PAD_BYTES].zero_()
        r, olen, _ = ctx.inflate_raw(comp.data_ptr(), cb, dec.data_ptr(), dec.numel(), DEV | ndfl.IN_PADDED)
        t2 = time.perf_counter()
        st.update(eb=eb, cb=cb, r=r, olen=olen, ti=ctx.timings()["inflate_span"], wc=t1 - t, wi=t2 - t1)
    dt = timed(run, 2)
    ok = st["r"] == 0 and st["olen"] == n and torch.equal(dec[:n], data)
    v = verify_stream(data, None, True, comp, st["eb"], 16)
    cb = st["cb"]
    return {"config": "c5: RLE_DYNAMIC round trip of 16 GiB random+repeat (device-resident, one GPU)",
            "bytes": n, "round_trip_ok": ok, "bit_exact": v["bit_exact"], "verify": v,
            "ratio": round(cb / n, 4), "ms_per_round_trip": round(dt * 1e3, 2),
            "input_MiBps": round((n + cb) / dt / MIB, 1),
            "compress_ms": round(st["td"], 2), "compress_wall_ms": round(st["wc"] * 1e3, 2),
            "inflate_span_ms": round(st["ti"], 2), "inflate_wall_ms": round(st["wi"] * 1e3, 2),
            "compress_frac_hbm": round((n + cb) / (st["td"] / 1e3) / 8e12, 4),
            "decompress_frac_hbm": round((n + cb) / (st["ti"] / 1e3) / 8e12, 4),
            "decompress_read_frac_hbm": round(cb / (st["ti"] / 1e3) / 8e12, 4),
            "round_trip_frac_hbm": round(2 * (n + cb) / dt / 8e12, 4), "corpus_gen_s": round(gen_s, 1)}


def main():
    which = sys.argv[1:] or ["c1", "c2", "c3", "c5"]
    ctx = ndfl.Context(0)
    for w in which:
        t = time.perf_counter()
        r = globals()[w](ctx)
        r["wall_s"] = round(time.perf_counter() - t, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
