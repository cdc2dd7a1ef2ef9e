"""Round-6 probe (measurement tooling, not product code): decode N bytes of the bench corpus with
the flat groups on and off (NDFL_FLAT, read when a context is created) and print the timings; run
with NDFL_STATS=1 for the library's per-pass counters on stderr.
Usage: python scripts/r06/flat_probe.py [MiB] [flat...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import ndfl  # noqa: E402
import corpus  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
flats = sys.argv[2:] or ["1", "0"]
n = mib << 20
if os.environ.get("PROBE_DATA") == "random":   # incompressible data only: the flat groups alone
    data = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=torch.Generator("cuda").manual_seed(3))
else:
    data = corpus.c4_mixed(n, seed=0xC4, device="cuda")
L = ndfl._lib.load()
cap = L.ndfl_deflate_bound(n, 65536) + 64
comp = torch.zeros(cap + 256, dtype=torch.uint8, device="cuda")
dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
for f in flats:
    os.environ["NDFL_FLAT"] = f
    ctx = ndfl.Context(0)
    eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, D)
    for rep in range(2):
        torch.cuda.synchronize()
        r, olen, bits = ctx.inflate_raw(comp.data_ptr(), (eb + 7) // 8, dec.data_ptr(), dec.numel(), D)
        ok = r == 0 and olen == n and bool(torch.equal(dec[:n], data))
        t = ctx.timings()
        print(f"flat={f} rep={rep}: ok {ok} find {t['inflate_find']:.3f} count {t['inflate_count']:.3f} "
              f"emit {t['inflate_emit']:.3f} span {t['inflate_span']:.3f} flat chains {int(t['inflate_flat_chains'])} "
              f"of {int(t['inflate_candidates'])}", flush=True)
    del ctx
