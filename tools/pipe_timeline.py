#!/usr/bin/env python3
"""Per-frame GPU timeline of the pipelined host-buffer path from a rocprofv3 trace
(`--kernel-trace --memory-copy-trace`, csv) of tools/pipe_probe.py or bench.py's pcie legs.

    python tools/pipe_timeline.py <trace dir> [--last N]

A frame = one k_s1_prep launch (its kernels run k_s1_prep .. k_cnt_to_host on the compute stream);
its copy-in is the last host->device copy of >= 1 MB that ends before its k_s1_prep starts, its
copy-out the k_rows_to_host launch (or device->host copy) that starts after its k_cnt_to_host.
Prints, per frame (ms, relative to the first frame's copy-in start): copy-in start / end, kernels
start / end, copy-out start / end, the wait between the copy-in end and the first kernel, and the
period between consecutive frames' kernel starts.
"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--last", type=int, default=12)
    a = p.parse_args()
    kt = rows(a.trace, "*kernel_trace.csv")
    mc = rows(a.trace, "*memory_copy_trace.csv")
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                  r.get("Queue_Id"), r.get("Stream_Id")) for r in kt), key=lambda x: x[0])
    h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in mc
                 if "HOST_TO_DEVICE" in r["Direction"])
    d2h = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in mc
                 if "DEVICE_TO_HOST" in r["Direction"])
    frames = []
    for i, k in enumerate(ks):
        if "k_s1_prep" not in k[2]:
            continue
        end = None
        for k2 in ks[i:]:
            if "k_cnt_to_host" in k2[2]:
                end = k2
                break
        if end is None:
            continue
        cin = [c for c in h2d if c[1] <= k[0] and c[1] - c[0] > 200_000]
        cin = cin[-1] if cin else None
        out = [k2 for k2 in ks if "k_rows_to_host" in k2[2] and k2[0] >= end[1]]
        out = out[0] if out else None
        if out is None:
            o2 = [c for c in d2h if c[0] >= end[1]]
            out = (o2[0][0], o2[0][1], "d2h") if o2 else None
        frames.append((cin, k, end, out))
    frames = frames[-a.last:]
    if not frames:
        print("no frames found")
        return
    t0 = frames[0][0][0] if frames[0][0] else frames[0][1][0]
    ms = lambda t: (t - t0) / 1e6   # noqa: E731
    print(f"{'in0':>8} {'in1':>8} {'k0':>8} {'k1':>8} {'out0':>8} {'out1':>8} {'wait':>6} "
          f"{'in_ms':>6} {'k_ms':>6} {'out_ms':>6} {'period':>7}")
    prev = None
    for cin, k, end, out in frames:
        i0, i1 = (ms(cin[0]), ms(cin[1])) if cin else (float("nan"),) * 2
        o0, o1 = (ms(out[0]), ms(out[1])) if out else (float("nan"),) * 2
        k0, k1 = ms(k[0]), ms(end[1])
        per = k0 - prev if prev is not None else float("nan")
        prev = k0
        print(f"{i0:8.3f} {i1:8.3f} {k0:8.3f} {k1:8.3f} {o0:8.3f} {o1:8.3f} {k0 - i1:6.3f} "
              f"{i1 - i0:6.3f} {k1 - k0:6.3f} {o1 - o0:6.3f} {per:7.3f}")


if __name__ == "__main__":
    main()
