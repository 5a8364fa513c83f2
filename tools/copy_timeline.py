#!/usr/bin/env python3
"""Kernels and memory copies of a rocprofv3 run (--kernel-trace --memory-copy-trace, csv) on one
time axis: the last `span_ms` milliseconds, each event's start offset, duration and queue.
    python tools/copy_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> [span_ms]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
span = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
ev = []
for f in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:48],
                   r.get("Queue_Id", r.get("Stream_Id", ""))))
for f in glob.glob(os.path.join(d, "**", "*_memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        nb = r.get("Bytes", r.get("Size", ""))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C",
                   "%s %s B" % (r.get("Direction", r.get("Operation", "")), nb), r.get("Stream_Id", "")))
ev.sort()
t_end = max(e[1] for e in ev)
t0 = t_end - span * 1e6
for s, e, k, name, q in ev:
    if e < t0:
        continue
    print("%9.3f ms %8.3f ms  %s  %-48s %s" % ((s - t0) / 1e6, (e - s) / 1e6, k, name, q))
