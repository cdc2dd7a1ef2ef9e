"""Round-6 strict-stage probe, one variant per process (measurement tooling, not product code):
compress the bench corpus (4 GiB config-4 mix, seed 0xC4) with the round-4 library given by
NDFL_LIB_PATH (scripts/r06/strict_probe/build.sh) and decode it with NDFL_STRICT_PROBE set, which
dumps every finder survivor with the strict stage's verdict (strict_probe.patch).
Usage: NDFL_LIB_PATH=... NDFL_STRICT_PROBE=out.bin python probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.join(HERE, "r4", "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import ndfl  # noqa: E402
import corpus  # noqa: E402

n = int(os.environ.get("PROBE_BYTES", str(4 << 30)))
data = corpus.c4_mixed(n, seed=0xC4, device="cuda")
ctx = ndfl.Context(0)
L = ndfl._lib.load()
cap = L.ndfl_deflate_bound(n, 65536) + 64
comp = torch.zeros(cap + 256, dtype=torch.uint8, device="cuda")
D = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
eb, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, 3, True, 0, comp.data_ptr(), cap, D)
dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
r, olen, bits = ctx.inflate_raw(comp.data_ptr(), (eb + 7) // 8, dec.data_ptr(), dec.numel(), D)
ok = r == 0 and olen == n and bool(torch.equal(dec[:n], data))
t = ctx.timings()
print(f"{os.path.basename(os.environ.get('NDFL_LIB_PATH', ''))}: code {r}, round trip {ok}, "
      f"candidates {int(t['inflate_candidates'])}, comp bytes {(eb + 7) // 8}", flush=True)
