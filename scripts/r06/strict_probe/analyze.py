"""Compare the strict stage's per-survivor verdicts of two probe dumps (good build first): which
survivors the good build accepts and the other does not, and what the other build did with them.
Verdict codes (strict_probe.patch): 0 never decided, 1 dynamic accepted, 2 dynamic rejected at the
end (bit 4: no end-of-block code, bit 5: literal Kraft sum != 1), 3 dynamic rejected midway (bits
4-13 symbols decoded i, 14-23 total, 24 bad repeat, 25 lit Kraft over, 26 dist Kraft over, 27 run
past total, 28 past the input), 4 stored accepted, 5 stored rejected, 6 incomplete code-length code."""
import collections
import sys

import numpy as np


def load(path):
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(4), dtype=np.uint32)[0])
        q = np.frombuffer(f.read(8 * n), dtype=np.uint64)
        v = np.frombuffer(f.read(4 * n), dtype=np.uint32)
    p = q & np.uint64((1 << 63) - 1)
    o = np.argsort(p, kind="stable")
    return p[o], v[o], (q[o] >> np.uint64(63)).astype(np.uint8)


def main():
    gp, gv, gd = load(sys.argv[1])
    for path in sys.argv[2:]:
        lp, lv, ld = load(path)
        same_set = len(gp) == len(lp) and bool(np.array_equal(gp, lp))
        print(f"== {path}: {len(lp)} survivors, same survivor set as the good build: {same_set}")
        if not same_set:
            continue
        gacc = (gv == 1) | (gv == 4)
        lacc = (lv == 1) | (lv == 4)
        print(f"   accepted: good {int(gacc.sum())}, this {int(lacc.sum())}; accepted here only {int((lacc & ~gacc).sum())}")
        lost = gacc & ~lacc
        codes = collections.Counter((lv[lost] & 15).tolist())
        print(f"   lost {int(lost.sum())}: verdicts here {dict(codes)} (0 = never decided)")
        kinds = collections.Counter(ld[lost].tolist())
        print(f"   lost by kind (1 = dynamic, 0 = stored): {dict(kinds)}")
        diff_all = gv != lv
        print(f"   survivors with a different verdict: {int(diff_all.sum())} of {len(lv)}; "
              f"undecided here: {int((lv == 0).sum())}, undecided in the good build: {int((gv == 0).sum())}")
        ex = np.nonzero(lost)[0][:12]
        for k in ex:
            x = int(lv[k])
            det = ""
            if (x & 15) == 3:
                det = (f" i={(x >> 4) & 1023} total={(x >> 14) & 1023} bad={(x >> 24) & 1} litover={(x >> 25) & 1} "
                       f"distover={(x >> 26) & 1} runpast={(x >> 27) & 1} pastinput={(x >> 28) & 1}")
            print(f"   p={int(lp[k])} kind={int(ld[k])} good={int(gv[k])} here={x & 15}{det}")


if __name__ == "__main__":
    main()
