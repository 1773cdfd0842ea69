#!/usr/bin/env python3
"""Raw kernel + copy events of a rocprofv3 csv trace around one frame of the pipelined path
(ms relative to the k-th last >= 0.5 ms host->device copy).
    python tools/trace_dump.py <trace dir> [k=12] [span_ms=7.5]"""
import csv
import glob
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
span = float(sys.argv[3]) if len(sys.argv) > 3 else 7.5
kt = list(csv.DictReader(open(glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0])))
mc = list(csv.DictReader(open(glob.glob(d + '/**/*memory_copy_trace.csv', recursive=True)[0])))
ev = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K q%s s%s' % (r['Queue_Id'], r['Stream_Id']),
       r['Kernel_Name'].split('(')[0].split('::')[-1][:40]) for r in kt]
ev += [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C s%s' % r['Stream_Id'], r['Direction'][12:])
       for r in mc]
ev.sort()
big = [e for e in ev if e[2].startswith('C') and e[1] - e[0] > 500000 and 'HOST_TO' in e[3]]
t0 = big[-k][0]
for e in ev:
    if t0 - 0.3e6 <= e[0] <= t0 + span * 1e6:
        print('%8.3f %8.3f %7.3f %-10s %s' % ((e[0] - t0) / 1e6, (e[1] - t0) / 1e6, (e[1] - e[0]) / 1e6,
                                             e[2], e[3]))
