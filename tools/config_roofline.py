#!/usr/bin/env python3
"""Roofline lines for BASELINE.json configs 2-5 from a tools/bench_tracker.py
line and the rocprofv3 kernel stats of the same command.

    python tools/config_roofline.py BENCH.json KERNEL_STATS.csv [FETCH_DIR WRITE_DIR] > line.json

Two views, both printed:
  * canonical: §8(d)'s per-update algorithmic bytes B and FLOPs F (dense formulation: a 16*N*M
    cost matrix, the full Kalman state, the D=512 cosine GEMMs), bound = max(B / 8 TB/s,
    F / f64 peak) per update, and the fraction of it the measured update time reaches;
  * per kernel: every kernel's share of the step, with its own bound where it has one (the f64
    embedding GEMMs: FLOPs / duration vs the f64 peak; the dense cost passes: bytes / duration vs
    HBM); the first-round solves (k_*_lap) and the one-block association kernels are dependent
    chains (Dijkstra steps, list scans) and carry no roofline ("latency").
With the FETCH_SIZE / WRITE_SIZE passes of the same command (rocprofv3 --pmc, separate runs), every
kernel line also carries its measured HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB ->
bytes: MI355X_MICROARCH.md's gfx950 correction, as profiles/summarize.py) next to the algorithmic
bytes.  No line prints a fraction above 1: a kernel whose algorithmic bytes over its duration
exceed the HBM peak read operands another kernel wrote just before, and the 256-MiB Infinity Cache
(MALL) served them; such a line is labelled bound "cache" and its HBM fraction comes from the
counter bytes (or is null without counters).
Peaks: HBM 8.0 TB/s (MI355X_MICROARCH.md); f64 78.6 TFLOP/s (vector = matrix on MI355X, vendor
spec, SURVEY.md §8(d) -- not in the microarchitecture guide's measured table); the GEMM lines
also carry the fraction of the f64 MFMA rate measured on the box (49.6 TFLOP/s, 8 independent
v_mfma_f64_16x16x4_f64 chains per wave, tools/mfma_f64_peak.hip).
"""
import collections
import csv
import glob
import json
import os
import sys

HBM = 8.0e12
F64 = 78.6e12
F64_MEASURED = 49.6e12    # tools/mfma_f64_peak.hip on the box: profiles/r03ze_mfma_f64_peak.jsonl
STATE = {"ocsort": 448, "botsort": 576, "deepocsort": 576, "hybridsort": 720}
GEMMS = {"ocsort": 0, "botsort": 1, "deepocsort": 1, "hybridsort": 2}


def canonical(tracker, N, M, D):
    """SURVEY.md §8(d) 'Algorithmic bytes per update' and FLOPs, one stream."""
    S = STATE[tracker]
    b = 4 * S * N + 56 * M + 16 * N * M + 64 * N
    if tracker == "ocsort":
        b += 136 * N
    elif tracker == "botsort":
        b += 4 * D * (N + M) + 8 * D * N
    elif tracker == "deepocsort":
        b += 2 * S * N + 16 * N * M + 136 * N + 8 * D * N + 4 * D * M + 16 * D * N
    elif tracker == "hybridsort":
        b += 208 * N + 8 * D * N + 4 * D * 30 * N + 4 * D * M + 16 * D * N + 4 * D * N
    return b, 2 * N * M * D * GEMMS[tracker]


def kernel_model(tracker, name, trk, det, D, S):
    """Work of one launch summed over the streams (trk / det: live trackers / kept detections of
    the last frame, summed over streams): ('flop', F) for the embedding GEMMs, ('hbm', B) for the
    dense cost passes (each f64 matrix entry read / written once), None for latency chains."""
    nm = trk * det / S   # matrix entries over all streams (the streams are alike: S * (trk/S) * (det/S))
    if "_emb" in name and tracker in ("deepocsort", "hybridsort"):
        return ("flop", 2.0 * nm * D)
    if tracker == "ocsort" and "k_oc_cost" in name:
        return ("hbm", 2 * 8 * nm)            # asso + asso+angle written
    if tracker == "deepocsort":
        if "k_doc_cost" in name:
            return ("hbm", 2 * 8 * nm)
        if "k_doc_final" in name:
            return ("hbm", 4 * 8 * nm)        # asso, emb, cost read; cost written
        if "k_doc_aw" in name and "cols" not in name:
            return ("hbm", 2 * 8 * nm)        # emb read by rows and by column chunks
    if "rowpre" in name:
        return ("hbm", 8 * nm)
    return None


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]


def pmc_means(d, counter):
    """Per kernel: the counter's mean per dispatch (rocprofv3 --pmc CSV under d), or {}."""
    if not d:
        return {}
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in agg.items() if v}


def main():
    bench = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    rows = list(csv.DictReader(open(sys.argv[2])))
    fetch = pmc_means(sys.argv[3] if len(sys.argv) > 3 else None, "FETCH_SIZE")
    write = pmc_means(sys.argv[4] if len(sys.argv) > 4 else None, "WRITE_SIZE")
    tracker = bench["metric"].split()[0]
    N = int(bench["metric"].split("@")[1].split()[0])
    D = int(bench["config"]["workload"].split("D=")[1].split(",")[0]) if "D=" in bench["config"]["workload"] else 0
    S = int(bench["config"]["streams"])
    Q = int(bench["config"].get("queues", 1))
    fc = bench.get("frame_counts", {})
    trk = fc.get("trackers", N * S)
    det = fc.get("high", N * S)
    B, F = canonical(tracker, N, N, D)
    t_upd = bench["ms_per_step"] * 1e-3 / S
    tb, tf = B / HBM, F / F64
    bound = max(tb, tf)
    kernels = []
    steps = bench["steps"] + bench["warmup"]
    for r in rows:
        name = r["Name"]
        if "yta::" not in name:
            continue
        avg = float(r["AverageNs"]) * 1e-9
        calls = int(r["Calls"])
        kn = short(name)
        k = {"kernel": kn, "avg_us": round(avg * 1e6, 2), "calls": calls,
             "share_of_step": round(avg * calls / steps / (bench["ms_per_step"] * 1e-3), 4)}
        cb = None
        if kn in fetch and kn in write:    # measured HBM bytes per launch (gfx950: FETCH x 2)
            cb = (2 * fetch[kn] + write[kn]) * 1024
            k.update(counter_bytes=round(cb), counter_gbs=round(cb / avg / 1e9, 1),
                     counter_frac=round(cb / avg / HBM, 4))
        m = kernel_model(tracker, name, trk, det, D, S)
        if m is not None and Q > 1:       # Q engines: one launch covers S / Q of the streams
            m = (m[0], m[1] / Q)
        if m is None:
            k["bound"] = "latency"
        elif m[0] == "flop":
            k.update(bound="f64", achieved_tflops=round(m[1] / avg / 1e12, 2),
                     peak_tflops=F64 / 1e12, frac=round(m[1] / avg / F64, 4),
                     measured_peak_tflops=F64_MEASURED / 1e12,
                     frac_of_measured_peak=round(m[1] / avg / F64_MEASURED, 4))
        else:
            ach = m[1] / avg
            k.update(alg_bytes=round(m[1]), achieved_gbs=round(ach / 1e9, 1), peak_gbs=HBM / 1e9)
            if cb is not None:
                k["counter_over_alg"] = round(cb / m[1], 3)
            if ach <= HBM:
                k.update(bound="hbm", frac=round(ach / HBM, 4))
            else:   # operands written just before by another kernel, served from the MALL
                k.update(bound="cache", frac=(round(cb / avg / HBM, 4) if cb is not None
                                              and cb / avg <= HBM else None),
                         note="algorithmic bytes / duration exceed the HBM peak: the operands "
                              "come from the 256-MiB Infinity Cache; frac = measured HBM bytes "
                              "/ duration / peak")
        kernels.append(k)
    kernels.sort(key=lambda k: -k["share_of_step"])
    out = {"tracker": tracker, "config": bench["config"], "calls_per_s": bench["value"],
           "ms_per_update": t_upd * 1e3,
           "canonical": {"bytes_per_update": B, "flops_per_update": F,
                         "t_bytes_us": tb * 1e6, "t_flops_us": tf * 1e6,
                         "binding": "f64" if tf > tb else "hbm",
                         "bound_us": bound * 1e6, "frac": bound / t_upd},
           "dominant": kernels[0] if kernels else None, "kernels": kernels}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
