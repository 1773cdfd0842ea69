#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<tag>_summary.{json,md}.

    python profiles/summarize.py <tag> <kernel_trace_dir> [<fetch_pmc_dir> <write_pmc_dir>]

* kernel time: `*_kernel_stats.csv` of `rocprofv3 --kernel-trace --stats` (average ns per launch).
* HBM traffic: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (MI355X_MICROARCH.md
  §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
  wide coalesced read, so the read side is doubled; WRITE_SIZE is taken as is).  Per-launch
  averages per kernel name.
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.replace("yta::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def kernel_stats(d):
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    out = {}
    for r in csv.DictReader(open(f)):
        out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "total_pct": float(r["Percentage"])}
    return out


def pmc(d, counter):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag, kt = sys.argv[1], sys.argv[2]
    stats = kernel_stats(kt)
    if len(sys.argv) > 4:
        fetch, write = pmc(sys.argv[3], "FETCH_SIZE"), pmc(sys.argv[4], "WRITE_SIZE")
        for k, v in stats.items():
            if k in fetch and k in write:
                v["fetch_kib_raw"] = fetch[k]
                v["write_kib"] = write[k]
                v["hbm_bytes_corrected"] = (2 * fetch[k] + write[k]) * 1024
                v["hbm_gbs"] = v["hbm_bytes_corrected"] / (v["avg_us"] * 1e-6) / 1e9
    here = os.path.dirname(os.path.abspath(__file__))
    json.dump(stats, open(os.path.join(here, f"{tag}_summary.json"), "w"), indent=1)
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "| kernel | calls | avg µs | % time | HBM bytes/launch (2×FETCH+WRITE) | GB/s |",
             "|---|---|---|---|---|---|"]
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_pct"]):
        hb = v.get("hbm_bytes_corrected")
        lines.append(f"| {k} | {v['calls']} | {v['avg_us']:.2f} | {v['total_pct']:.2f} | "
                     f"{'%.3g' % hb if hb else '-'} | {'%.0f' % v['hbm_gbs'] if hb else '-'} |")
    open(os.path.join(here, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
