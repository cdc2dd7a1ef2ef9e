"""Diagnose GPU inflate of LZ77-heavy streams (GPU FULL_DYNAMIC and zlib) at growing sizes."""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ndfl  # noqa: E402
import corpus  # noqa: E402

ctx = ndfl.Context(0)
sizes = [int(x) for x in (sys.argv[1:] or ["8", "32", "128"])]
for mib in sizes:
    data = corpus.c3_text(mib << 20, seed=7).numpy().tobytes()
    for kind in ["gpu_full", "zlib6"]:
        comp = ctx.deflate(data, "FULL_DYNAMIC") if kind == "gpu_full" else zlib.compressobj(6, zlib.DEFLATED, -15).compress(data) + b""
        if kind == "zlib6":
            co = zlib.compressobj(6, zlib.DEFLATED, -15)
            comp = co.compress(data) + co.flush()
        t = time.time()
        r, olen, bits = ctx.inflate_raw(*(lambda b: (b[1], len(comp)))(( None, __import__('ctypes').addressof(src := __import__('ctypes').create_string_buffer(comp, len(comp))))),
                                        __import__('ctypes').addressof(dst := __import__('ctypes').create_string_buffer(len(data) + 16)), len(data) + 16, 0)
        dt = time.time() - t
        good = dst.raw[:olen] == data[:olen]
        first_bad = -1
        if not good:
            out = dst.raw[:olen]
            first_bad = next(i for i in range(olen) if out[i] != data[i])
        print(f"{mib} MiB {kind}: comp {len(comp)} code {r} out_len {olen}/{len(data)} prefix_ok {good} "
              f"first_bad {first_bad} {dt*1e3:.0f} ms timings {ctx.timings()}", flush=True)
