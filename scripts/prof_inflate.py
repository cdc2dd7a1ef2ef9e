"""Profiling driver: compress 1 GiB of the c4 corpus once, then decompress it (device buffers)."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch, ndfl, corpus
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 30)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
x = corpus.c4_mixed(n, device="cuda")
ctx = ndfl.Context(0)
L = ndfl._lib.load()
cap = L.ndfl_deflate_bound(n, 65536) + 64
comp = torch.empty(cap, dtype=torch.uint8, device="cuda")
dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
for _ in range(reps):
    eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, x.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, D)
    r, olen, bits = ctx.inflate_raw(comp.data_ptr(), (eb + 7) // 8, dec.data_ptr(), dec.numel(), D)
    assert r == 0 and olen == n
print(ctx.timings(), flush=True)
