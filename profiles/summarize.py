#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<tag>_summary.{json,md} (+ roofline_traffic.json).

    python profiles/summarize.py <tag> <kernel_trace_dir> <fetch_pmc_dir> <write_pmc_dir> \
        [--streams S] [--n N] [--bench-json FILE]

* kernel time: `*_kernel_stats.csv` of `rocprofv3 --kernel-trace --stats` (average ns per launch).
* HBM traffic: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (MI355X_MICROARCH.md
  §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
  wide coalesced read, so the read side is doubled; WRITE_SIZE is taken as is).  Per-launch
  averages per kernel name.
* roofline_traffic.json: the HBM bytes per launch of the roofline kernel (k_apply) with the
  workload they were measured on; bench.py reports them as `roofline.traffic` when its own
  workload matches.
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    n = name.replace("yta::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def kernel_stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "total_pct": float(r["Percentage"])}
    return out, f


def pmc(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("kt")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--streams", type=int, default=None)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--queues", type=int, default=1, help="engines (HIP streams) of the run")
    ap.add_argument("--steps", type=int, default=None,
                    help="frames per engine in the profiled run (for the per-step traffic)")
    ap.add_argument("--bench-json", default=None)
    args = ap.parse_args()
    here = os.path.dirname(os.path.abspath(__file__))
    stats, ks_file = kernel_stats(args.kt)
    fetch, write = pmc(args.fetch, "FETCH_SIZE"), pmc(args.write, "WRITE_SIZE")
    for k, v in stats.items():
        if k in fetch and k in write:
            v["fetch_kib_raw"] = fetch[k]
            v["write_kib"] = write[k]
            v["hbm_bytes_corrected"] = (2 * fetch[k] + write[k]) * 1024
            v["hbm_gbs"] = v["hbm_bytes_corrected"] / (v["avg_us"] * 1e-6) / 1e9
    summary = {"tag": args.tag, "streams": args.streams, "n": args.n, "kernels": stats}
    if args.bench_json and os.path.exists(args.bench_json):
        lines = [l for l in open(args.bench_json).read().splitlines() if l.startswith("{")]
        if lines:
            summary["bench"] = json.loads(lines[-1])
    json.dump(summary, open(os.path.join(here, f"{args.tag}_summary.json"), "w"), indent=1)
    os.system(f"cp '{ks_file}' '{os.path.join(here, args.tag + '_kernel_stats.csv')}'")
    lines = [f"# rocprofv3 summary `{args.tag}`", "",
             f"Workload: bench.py --streams {args.streams} --queues {args.queues}, {args.n} tracks x "
             f"{args.n} dets per stream.  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), separate passes.",
             "",
             "| kernel | calls | avg µs | % time | HBM bytes/launch | GB/s |",
             "|---|---|---|---|---|---|"]
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_pct"]):
        hb = v.get("hbm_bytes_corrected")
        lines.append(f"| {k} | {v['calls']} | {v['avg_us']:.2f} | {v['total_pct']:.2f} | "
                     f"{'%.4g' % hb if hb else '-'} | {'%.0f' % v['hbm_gbs'] if hb else '-'} |")
    open(os.path.join(here, f"{args.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    ka = next((k for k in stats if k.split("<")[0] == "k_apply"), None)
    if ka and "hbm_bytes_corrected" in stats[ka]:
        # per step: every tracker kernel once per engine (the k_* launches of a frame)
        step = sum(v["hbm_bytes_corrected"] for k, v in stats.items()
                   if k.startswith("k_") and k != "k_reset" and "hbm_bytes_corrected" in v)
        json.dump({"tag": args.tag, "streams": args.streams, "n": args.n, "queues": args.queues,
                   "kernel": "k_apply",
                   "hbm_bytes_per_launch": stats[ka]["hbm_bytes_corrected"],
                   "hbm_bytes_per_step": step * args.queues,
                   "avg_us_rocprof": stats[ka]["avg_us"]},
                  open(os.path.join(here, "roofline_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
