"""Time the LZ77 (FULL_DYNAMIC) encoder on the config-3 text corpus, device-resident in and out."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import ndfl  # noqa: E402
import corpus  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=int, default=1024)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--check-mib", type=int, default=0, help="compare the first N MiB against the oracle")
args = ap.parse_args()
n = args.mib << 20
data = corpus.c3_text(n, device="cuda")
ctx = ndfl.Context(0)
cap = ndfl.load().ndfl_deflate_bound(n, 65536) + 64
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
flags = ndfl.IN_DEVICE | ndfl.OUT_DEVICE
for r in range(args.reps):
    torch.cuda.synchronize()
    t = time.time()
    endbits, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), n, 65536, ndfl.Lz77Huffman.FULL_DYNAMIC,
                                        True, 0, out.data_ptr(), cap, flags)
    torch.cuda.synchronize()
    dt = time.time() - t
    print(f"rep {r}: {dt*1e3:.1f} ms wall, kernels {ctx.last_kernel_ms():.1f} ms, {n / dt / 2**20:.0f} MiB/s, "
          f"ratio {endbits / 8 / n:.4f}", flush=True)
comp = out[:(endbits + 7) // 8].cpu().numpy().tobytes()
reason, dec, _ = ctx.inflate(comp, out_cap=n + 16)
assert reason is None and dec == data.cpu().numpy().tobytes(), "round trip failed"
print("round trip ok")
if args.check_mib:
    import oracle_lib as O
    m = args.check_mib << 20
    host = data[:m].cpu().numpy().tobytes()
    got = ctx.deflate(host, "FULL_DYNAMIC")
    assert got == O.deflate(host, "FULL_DYNAMIC"), "oracle mismatch"
    print(f"oracle parity ok on {args.check_mib} MiB")
