"""One-off check: a single ndfl_inflate call whose output exceeds 4 GiB (c4 mix, 4.5 GiB)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import ndfl  # noqa: E402
import corpus  # noqa: E402

n = (4 << 30) + (512 << 20)
data = corpus.c4_mixed(n, seed=7, device="cuda")
ctx = ndfl.Context(0)
cap = ndfl._lib.load().ndfl_deflate_bound(n, 65536) + 64
comp = torch.empty(cap, dtype=torch.uint8, device="cuda")
DEV = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, DEV)
cb = (eb + 7) // 8
dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
t = time.time()
r, olen, _ = ctx.inflate_raw(comp.data_ptr(), cb, dec.data_ptr(), dec.numel(), DEV)
torch.cuda.synchronize()
print(f"inflate of {olen} bytes (> 4 GiB): code {r}, {time.time() - t:.3f} s, exact {olen == n and torch.equal(dec[:n], data)}")
