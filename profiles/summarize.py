#!/usr/bin/env python3
"""Condense one collect.sh run into committed summaries (profiles/TAG_*):
  TAG_bench.json          the bench line;           TAG_breakdown.txt  its HIP-event per-kernel breakdown
  TAG_kernel_stats.csv    rocprofv3 --stats summary (all kernels of the short bench run)
  TAG_c3_pmc.json / TAG_c4_pmc.json   the same for the C3 line (block level walk) and the C4 line; TAG_c3_bench.json / TAG_c4_bench.json /
                          TAG_cpu_full.json   the secondary lines
  TAG_pmc.json            per kernel (rocprof name + grid): mean FETCH_SIZE / WRITE_SIZE per dispatch (KB as
                          rocprofv3 reports them) and dispatch counts, plus the 4-byte streaming-read calibration
                          measured on k_radix_hist (reads exactly units*4 key bytes, coalesced 4 B/lane).
Usage: summarize.py OUT_DIR TAG
"""
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _find(d, name):
    hits = glob.glob(os.path.join(d, "**", name), recursive=True)
    return hits[0] if hits else None


def _short(name):
    return name.split("(")[0].replace("void ", "")


def pmc(d, counter):
    f = _find(d, "*counter_collection.csv")
    out = {}
    if not f:
        return out
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            k = "%s grid=%s" % (_short(r["Kernel_Name"]), r["Grid_Size"])
            s = out.setdefault(k, [0.0, 0])
            s[0] += float(r["Counter_Value"])
            s[1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in out.items()}


def calibration(res):
    """k_radix_hist reads n keys (4 B each, coalesced 4 B/lane) and writes 1 KB/tile: FETCH_SIZE per algorithmic byte
    of its largest batch-sized dispatch (the largest ratio over dispatches of >= 2^20 keys)."""
    cal = None
    for k, e in res.items():
        if k.startswith("ad::k_radix_hist") and "FETCH_SIZE_KB_mean" in e:
            grid = int(k.split("grid=")[1])
            n_keys = grid // 256 * 4096          # full tiles; the last tile may be partial (upper bound)
            if n_keys >= (1 << 20):
                ratio = e["FETCH_SIZE_KB_mean"] * 1024 / (n_keys * 4)
                if cal is None or ratio > cal["fetch_per_alg_byte"]:
                    cal = {"kernel": k, "alg_read_bytes": n_keys * 4, "fetch_per_alg_byte": ratio}
    return cal


def main():
    out, tag = sys.argv[1], sys.argv[2]
    dst = lambda s: os.path.join(HERE, "%s_%s" % (tag, s))
    if os.path.exists(os.path.join(out, "bench.json")):
        shutil.copy(os.path.join(out, "bench.json"), dst("bench.json"))
    if os.path.exists(os.path.join(out, "bench.err")):
        with open(os.path.join(out, "bench.err")) as f:
            lines = [l for l in f if l.startswith("  ")]
        with open(dst("breakdown.txt"), "w") as f:
            f.writelines(lines)
    ks = _find(os.path.join(out, "stats"), "*kernel_stats.csv")
    if ks:
        shutil.copy(ks, dst("kernel_stats.csv"))
    fetch = pmc(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = pmc(os.path.join(out, "write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        e = {}
        if k in fetch:
            e["FETCH_SIZE_KB_mean"], e["dispatches"] = fetch[k]
        if k in write:
            e["WRITE_SIZE_KB_mean"] = write[k][0]
            e.setdefault("dispatches", write[k][1])
        res[k] = e
    cal = calibration(res)
    doc = {"note": "FETCH_SIZE/WRITE_SIZE per dispatch in KB (1 KB = 1024 B) as rocprofv3 reports them on gfx950; "
                   "Infinity-Cache hits are counted (MI355X_MICROARCH.md, HBM section). Separate passes per counter.",
           "calibration_4B_stream_read": cal, "kernels": res}
    with open(dst("pmc.json"), "w") as f:
        json.dump(doc, f, indent=1)
    # C3's and C4's passes (collect.sh steps 6, 7): per kernel as above, each with its own calibration
    for cfg, what in (("c3", "C3 (1M Zipf txns)"), ("c4", "C4 (4M mixed key + range txns)")):
        fx, wx = pmc(os.path.join(out, cfg + "fetch"), "FETCH_SIZE"), pmc(os.path.join(out, cfg + "write"), "WRITE_SIZE")
        if not (fx or wx):
            continue
        rx = {}
        for k in sorted(set(fx) | set(wx)):
            e = {}
            if k in fx:
                e["FETCH_SIZE_KB_mean"], e["dispatches"] = fx[k]
            if k in wx:
                e["WRITE_SIZE_KB_mean"] = wx[k][0]
                e.setdefault("dispatches", wx[k][1])
            rx[k] = e
        with open(dst(cfg + "_pmc.json"), "w") as f:
            json.dump({"note": doc["note"] + " %s, bench.py --config %s --steps 1 --warmup 1." % (what, cfg.upper()),
                       "calibration_4B_stream_read": calibration(rx), "kernels": rx}, f, indent=1)
    for name in ("c3.json", "c4.json", "cpu_full.json"):
        if os.path.exists(os.path.join(out, name)):
            shutil.copy(os.path.join(out, name), dst(name.replace(".json", "_bench.json") if name != "cpu_full.json" else name))
    print("wrote", [os.path.basename(p) for p in glob.glob(os.path.join(HERE, tag + "_*"))])


if __name__ == "__main__":
    main()
