"""Per-kernel statistics from a rocprofv3 SQLite output (run_results.db) or kernel-trace CSV, split into the bench's
workload blocks (C2, C4, C5, in launch order) by the dispatch-order position of each launch:
    python tools/rocpd_stats.py <db> [n_blocks]"""
import csv
import sqlite3
import sys


def load(path):
    """(name, start ns, end ns) of every dispatch, by start: a rocprofv3 SQLite output or its
    --output-format csv kernel trace (*_kernel_trace.csv)"""
    if path.endswith(".csv"):
        rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))]
        return sorted(rows, key=lambda r: r[1])
    return list(sqlite3.connect(path).execute("select name, start, end from kernels order by start"))
from collections import defaultdict

db = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = load(db)
n = len(rows)
# block boundaries: equal share of the index-kernel launches (one per evaluation and block)
marks = [i for i, r in enumerate(rows) if r[0].startswith("mxp_index_dtp_")]
bounds = [0]
if nb > 1 and marks:
    per = len(marks) // nb
    bounds += [marks[per * b] for b in range(1, nb)]
bounds.append(n)
for b in range(nb):
    agg = defaultdict(list)
    for name, s, e in rows[bounds[b]:bounds[b + 1]]:
        agg[name].append((e - s) / 1000.0)
    print("== block %d (launches %d..%d)" % (b, bounds[b], bounds[b + 1]))
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:14]:
        d.sort()
        print("  %-40s n=%4d avg %8.2f us  med %8.2f us  sum %7.2f ms" % (name[:40], len(d), sum(d) / len(d), d[len(d) // 2], sum(d) / 1e3))
