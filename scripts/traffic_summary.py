"""Per-launch HBM traffic of each ndfl kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as calibrated on gfx950 (profiles/r06_fetch_calib.txt, scripts/r06/fetch_calib.hip: kernels
that move a known 2 GiB past the Infinity Cache in one access shape each):
  * FETCH_SIZE / WRITE_SIZE are in KiB per dispatch;
  * FETCH_SIZE reports exactly 1/2 of the bytes of a coalesced streaming read in every shape the ndfl
    kernels use -- 4-B/lane dword loads, 16-B/lane loads and LDS-DMA dword loads (one 256-B row per
    wave instruction) alike -> x2 for every kernel whose reads are such rows (all of the decoder's
    full-stream passes: finder ld4 groups, round staging by LDS-DMA, record and table loads);
  * WRITE_SIZE is exact for coalesced 4-B and 16-B stores; 16-B stores from 64 scattered lane cursors
    (the emit pass's output) read 2.8-2.9x the bytes written (partial lines leave L2): reported as
    measured, with that note.
Usage: python scripts/traffic_summary.py FETCH.csv WRITE.csv OUT.json"""
import collections
import csv
import json
import sys

# FETCH_SIZE correction per kernel (all calibrated shapes read at 1/2)
FETCH_CORR = collections.defaultdict(lambda: 2.0)
NOTES = {
    "ndfl_deflate_hist_kernel": "16-B/lane loads of the chunk (x2) plus the L2 touch of the next generation's "
                                "chunk (one byte per 128-B line; those lines are then read from L2 by the next "
                                "workgroup, so the pair counts each line about once); writes: 1.25 KiB per chunk",
    "ndfl_deflate_emit_kernel": "as hist: 16-B/lane chunk loads (x2) + the L2 touch; 4-B code-record loads; "
                                "coalesced 4-B interior stores (exact)",
    "ndfl_inflate_find_compact_kernel": "16-B/lane row loads of the stream (x2)",
    "ndfl_inflate_strict_kernel": "16-B/lane window loads of the survivors' bits (x2; gathered rows)",
    "ndfl_inflate_count_wave_kernel": "LDS-DMA dword rows of each round (x2), header records, candidate cursor; "
                                      "writes: segment records, table records, per-wave phase slots, scratch spills",
    "ndfl_inflate_emit_fast_kernel": "LDS-DMA dword rows of each round (x2), segment and table records (x2); writes "
                                     "are 16-B stores at 64 lane cursors: WRITE_SIZE 2.8-2.9x the bytes by "
                                     "calibration (profiles/r06_fetch_calib.txt), reported as measured",
    "ndfl_inflate_emit_wave_kernel": "as emit_fast; stores at 64 lane cursors (WRITE_SIZE above the bytes written)",
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
        corr = FETCH_CORR[k]
        out[k] = {"launches": nf, "fetch_bytes_raw": round(fb), "fetch_bytes": round(fb * corr),
                  "fetch_correction": corr, "write_bytes": round(wb), "traffic_bytes": round(fb * corr + wb),
                  "note": NOTES.get(k, "")}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in out.items():
        print(f"{k:34s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
