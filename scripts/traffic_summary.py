"""Per-launch HBM traffic of each ndfl kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3) prescribes:
  * FETCH_SIZE / WRITE_SIZE are in KiB per dispatch;
  * gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read -> x2 for
    the kernels whose input side is such a read (deflate_chunks: 16-B loads of the raw bytes);
  * WRITE_SIZE is exact for 16-B-per-lane streaming stores; other widths are uncalibrated (noted).
Usage: python scripts/traffic_summary.py FETCH.csv WRITE.csv OUT.json"""
import collections
import csv
import json
import sys

WIDE_READ = {"ndfl_deflate_chunks_kernel": True}
NOTES = {
    "ndfl_deflate_chunks_kernel": "16-B/lane streaming loads (x2 applied) and 16-B/lane interior stores: calibrated",
    "ndfl_deflate_hist_kernel": "raw: the chunk arrives partly through the previous generation's L2 touch (1-B "
                                "loads, one per 128-B line: counted in full) and partly through 16-B/lane loads "
                                "(counted half), so no single correction applies; raw = N (0.5 + 0.5 p) gives the "
                                "touched share p, and the actual fetch is about N; writes: 1.25 KiB per chunk",
    "ndfl_deflate_emit_kernel": "raw, as for hist (L2 touch + 16-B/lane loads; the 4-B code-record loads add "
                                "~1.7 KiB per chunk); 4-B/lane coalesced interior stores",
    "ndfl_inflate_emit_wave_kernel": "reads are 16-B prefetch per chain (uncalibrated, raw); stores are 4-B per lane "
                                     "at 64 independent chain cursors: partial lines leave L2 before they fill",
}


def load(path):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k], len(disp[k])) for k in tot}


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("ndfl"):
            continue
        f, nf = fetch.get(k, (0.0, 1))
        w, nw = write.get(k, (0.0, 1))
        fb = f * 1024 / max(nf, 1)
        wb = w * 1024 / max(nw, 1)
        corr = 2.0 if WIDE_READ.get(k) else 1.0
        out[k] = {"launches": nf, "fetch_bytes_raw": round(fb), "fetch_bytes": round(fb * corr),
                  "fetch_correction": corr, "write_bytes": round(wb), "traffic_bytes": round(fb * corr + wb),
                  "note": NOTES.get(k, "")}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in out.items():
        print(f"{k:34s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
