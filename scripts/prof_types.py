"""Per-data-type decode profile: compress n bytes of each c4 component alone, decompress twice,
print the library's phase timings (ms) and the compressed ratio."""
import sys, os, math
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch, ndfl, corpus
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 28)
g = torch.Generator(device="cuda").manual_seed(7)
gens = {
    "text": lambda: corpus._text(g, n, "cuda"),
    "binary": lambda: corpus._binary(g, n, "cuda"),
    "random": lambda: torch.randint(0, 256, (n,), generator=g, device="cuda", dtype=torch.uint8),
    "runs": lambda: corpus._runs(g, n, "cuda"),
}
ctx = ndfl.Context(0)
L = ndfl._lib.load()
D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
cap = L.ndfl_deflate_bound(n, 65536) + 64
comp = torch.empty(cap, dtype=torch.uint8, device="cuda")
dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else gens):
    x = gens[name]().contiguous()
    for _ in range(2):
        eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, x.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, D)
        r, olen, bits = ctx.inflate_raw(comp.data_ptr(), (eb + 7) // 8, dec.data_ptr(), dec.numel(), D)
        assert r == 0 and olen == n
    if not os.environ.get("NDFL_NOCHECK"):
        assert torch.equal(dec[:n], x)
    t = ctx.timings()
    print(f"{name:7s} ratio {eb / 8 / n:.3f} " + " ".join(f"{k}={v:.2f}" for k, v in t.items() if isinstance(v, float)), flush=True)
