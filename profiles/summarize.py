#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<tag>_summary.{json,md} (+ roofline_traffic.json).

    python profiles/summarize.py <tag> <kernel_trace_dir> <fetch_pmc_dir> <write_pmc_dir> \
        [--streams S] [--n N] [--bench-json FILE]

* kernel time: `*_kernel_stats.csv` of `rocprofv3 --kernel-trace --stats` (average ns per launch).
* HBM traffic: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes (MI355X_MICROARCH.md
  §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
  wide coalesced read, so the read side is doubled; WRITE_SIZE is taken as is).  Per-launch
  averages per kernel name.
* per-launch windows from the kernel trace (`*_kernel_trace.csv`, dispatch order per kernel
  name): with --pre P --steps K --queues Q --iso I (bench.py's untimed frames, timed frames,
  engines and isolated-leg frames), the first P*Q launches of a kernel are untimed, the next K*Q
  the timed region (engines overlapping), the last I the isolated leg (engine 0 alone).  The
  average duration and the PMC bytes are reported for the timed and the isolated windows.
* roofline_traffic.json: per kernel, the HBM bytes per isolated launch (and per timed launch) and
  the rocprof average durations, with the workload they were measured on; bench.py reports them
  in `roofline` / `per_kernel` when its own workload matches.
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


def base(name):
    return short(name).split("<")[0]


def windows(seq, pre, steps, queues, iso):
    """(timed, isolated) slices of one kernel's per-dispatch values in dispatch order."""
    if pre is None or steps is None:
        return seq, []
    n0, n1 = pre * queues, (pre + steps) * queues
    timed = seq[n0:n1]
    isolated = seq[n1:n1 + iso] if iso else []
    return timed, isolated


def mean(v):
    return sum(v) / len(v) if v else None


def trace(d):
    """Per kernel name: launch durations (us) in dispatch order, from the kernel trace."""
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not fs:
        return {}
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        rows[short(r["Kernel_Name"])].append(
            (int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return {k: [t for _, t in sorted(v)] for k, v in rows.items()}


def pmc(d, counter):
    """Per kernel name: the counter per dispatch, in dispatch order."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            k = short(r["Kernel_Name"])
            agg[k][int(r["Dispatch_Id"])] = agg[k].get(int(r["Dispatch_Id"]), 0.0) + float(
                r["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in agg.items()}


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
    ap.add_argument("--pre", type=int, default=None, help="untimed frames per engine")
    ap.add_argument("--iso", type=int, default=0, help="isolated-leg frames (engine 0 alone)")
    ap.add_argument("--bench-json", default=None)
    args = ap.parse_args()
    here = os.path.dirname(os.path.abspath(__file__))
    stats, ks_file = kernel_stats(args.kt)
    durs = trace(args.kt)
    fetch_all, write_all = pmc(args.fetch, "FETCH_SIZE"), pmc(args.write, "WRITE_SIZE")
    win = lambda seq: windows(seq, args.pre, args.steps, args.queues, args.iso)  # noqa: E731
    for k, v in stats.items():
        if k in durs:
            t, i = win(durs[k])
            v["avg_us_timed"], v["avg_us_isolated"] = mean(t), mean(i)
        if k in fetch_all and k in write_all:
            ft, fi = win(fetch_all[k])
            wt, wi = win(write_all[k])
            fetch, write = mean(fetch_all[k]), mean(write_all[k])
            v["fetch_kib_raw"] = fetch
            v["write_kib"] = write
            v["hbm_bytes_corrected"] = (2 * fetch + write) * 1024
            v["hbm_gbs"] = v["hbm_bytes_corrected"] / (v["avg_us"] * 1e-6) / 1e9
            if ft and wt:
                v["hbm_bytes_timed"] = (2 * mean(ft) + mean(wt)) * 1024
            if fi and wi:
                v["hbm_bytes_isolated"] = (2 * mean(fi) + mean(wi)) * 1024
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
             f"Windows per kernel (dispatch order): untimed {args.pre} x {args.queues}, timed "
             f"{args.steps} x {args.queues} (engines overlapping), isolated {args.iso} (engine 0 "
             "alone).",
             "",
             "| kernel | calls | avg µs (all) | avg µs timed | avg µs isolated | % time | "
             "HBM bytes/launch (all) | HBM bytes isolated | GB/s (all) |",
             "|---|---|---|---|---|---|---|---|---|"]
    f3 = lambda x, fmt: (fmt % x) if x else "-"  # noqa: E731
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_pct"]):
        hb = v.get("hbm_bytes_corrected")
        lines.append(f"| {k} | {v['calls']} | {v['avg_us']:.2f} | "
                     f"{f3(v.get('avg_us_timed'), '%.2f')} | "
                     f"{f3(v.get('avg_us_isolated'), '%.2f')} | {v['total_pct']:.2f} | "
                     f"{f3(hb, '%.4g')} | {f3(v.get('hbm_bytes_isolated'), '%.4g')} | "
                     f"{f3(v.get('hbm_gbs'), '%.0f')} |")
    open(os.path.join(here, f"{args.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    kern = {}
    for k, v in stats.items():
        if not k.startswith("k_") or "hbm_bytes_corrected" not in v:
            continue
        kern[base(k)] = {
            "name": k,
            "hbm_bytes_per_launch": v.get("hbm_bytes_isolated") or v["hbm_bytes_corrected"],
            "hbm_bytes_timed": v.get("hbm_bytes_timed"),
            "avg_us_isolated": v.get("avg_us_isolated"),
            "avg_us_timed": v.get("avg_us_timed"),
            "avg_us_all": v["avg_us"]}
    if "k_apply" in kern:
        # per step: every tracker kernel once per engine (the timed launches of a frame)
        step = sum((x["hbm_bytes_timed"] or x["hbm_bytes_per_launch"]) for x in kern.values()
                   if x["name"] != "k_reset")
        json.dump({"tag": args.tag, "streams": args.streams, "n": args.n, "queues": args.queues,
                   "note": "hbm_bytes_per_launch: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of the "
                           "isolated-leg launches (engine 0 alone) where the run had one, else "
                           "of every launch",
                   "kernels": kern, "hbm_bytes_per_step": step * args.queues},
                  open(os.path.join(here, "roofline_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
