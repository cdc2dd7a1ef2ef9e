"""Round 5 diagnostic: the decoder's accepted header set on the bench stream (4 GiB config-4 corpus,
RLE_DYNAMIC) for several builds of libndfl.so, e.g. strict stages at 3 / 4 / 5 waves per SIMD.
For each build: headers accepted, finder survivors, and for headers another build accepted but this
one did not: whether they were among this build's finder survivors (a strict-stage loss) or not (a
finder loss).  Usage: python scripts/r05/headers_ab.py [--size BYTES] lib1.so lib2.so ...
Each library runs in a child process (one library per process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(lib, size, out):
    os.environ["NDFL_LIB_PATH"] = lib
    sys.path.insert(0, os.path.join(ROOT, "deflate-library-java_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch
    import ndfl
    import corpus
    data = corpus.c4_mixed(size, seed=0xC4, device="cuda")
    torch.cuda.synchronize()
    ctx = ndfl.Context(0)
    L = ndfl._lib.load()
    cap = L.ndfl_deflate_bound(size, 65536) + 64
    comp = torch.zeros(cap + ndfl.IN_PAD_BYTES, dtype=torch.uint8, device="cuda")
    endbits, _ = ctx.deflate_chunks_raw(None, 0, 32768, data.data_ptr(), size, 65536, 3, True, 0, comp.data_ptr(),
                                        cap, ndfl.IN_DEVICE | ndfl.OUT_DEVICE)
    nbytes = (endbits + 7) // 8
    del data
    comp[nbytes:].zero_()
    torch.cuda.synchronize()
    runs = []
    for rep in range(3):
        hs, st, sv = ctx.inflate_headers_raw(comp.data_ptr(), nbytes, ndfl.IN_DEVICE | ndfl.IN_PADDED, survivors=True)
        runs.append({"headers": hs, "stats": st, "surv": sv})
    np.save(out + "_h.npy", np.array(runs[0]["headers"], dtype=np.uint64))
    np.save(out + "_s.npy", np.array([x & ~(1 << 63) for x in runs[0]["surv"]], dtype=np.uint64))
    print(json.dumps({"lib": os.path.basename(lib), "comp_bytes": nbytes,
                      "headers": [len(r["headers"]) for r in runs], "stats": [r["stats"] for r in runs],
                      "runs_identical": all(r["headers"] == runs[0]["headers"] for r in runs)}), flush=True)


def main():
    args = sys.argv[1:]
    size = 4 << 30
    if args and args[0] == "--size":
        size = int(args[1])
        args = args[2:]
    if args and args[0] == "--child":
        child(args[1], size, args[2])
        return
    import tempfile
    tmp = tempfile.mkdtemp()             # (the lists are ~70 MB each: kept out of gpurun_out)
    outs = []
    for lib in args:
        out = os.path.join(tmp, "hab_" + os.path.basename(lib).replace(".so", ""))
        rc = subprocess.call([sys.executable, "-u", __file__, "--size", str(size), "--child", lib, out],
                             timeout=600)
        if rc:
            sys.exit(rc)
        outs.append(out)
    import numpy as np
    sets = [set(np.load(o + "_h.npy").tolist()) for o in outs]
    union = set().union(*sets)
    for o, s in zip(outs, sets):
        sv = np.load(o + "_s.npy").tolist()
        index = {p: i for i, p in enumerate(sv)}
        lost = sorted(union - s)
        in_surv = sum(1 for p in lost if p in index)
        # where the lost headers sat in the strict stage's work list: slice = 128 consecutive survivors
        slices = {}
        for p in lost:
            if p in index:
                slices.setdefault(index[p] // 128, []).append(p)
        full = 0
        for sl, ps in slices.items():
            real = [q for q in sv[sl * 128:(sl + 1) * 128] if q in union]
            full += len(real) == len(ps)
        pos_in_slice = [index[p] % 128 for p in lost[:40] if p in index]
        print(json.dumps({"build": os.path.basename(o), "accepted": len(s), "missing_vs_union": len(lost),
                          "missing_in_own_survivors": in_surv, "slices_with_losses": len(slices),
                          "slices_all_real_lost": full, "first_missing": lost[:6],
                          "slot_in_slice": pos_in_slice,
                          "real_per_lossy_slice": [len([q for q in sv[sl * 128:(sl + 1) * 128] if q in union])
                                                   for sl in list(slices)[:20]],
                          "lost_per_lossy_slice": [len(v) for v in list(slices.values())[:20]]}), flush=True)


if __name__ == "__main__":
    main()
