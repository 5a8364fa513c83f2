"""One step's kernel timeline from a rocprofv3 SQLite output: the launches between two consecutive
launches of `anchor` (the step's first kernel), with their durations and the idle gaps between them.
    python tools/rocpd_timeline.py <db> [anchor] [which occurrence]"""
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

db = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "mxp_index_dtp_"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rows = load(db)
idx = [i for i, r in enumerate(rows) if r[0].startswith(anchor)]
a, b = idx[occ], idx[occ + 1]
t0 = rows[a][1]
prev_end = None
busy = 0
for name, s, e in rows[a:b]:
    gap = (s - prev_end) / 1000.0 if prev_end is not None else 0.0
    busy += e - s
    print("%9.2f us  +gap %6.2f  dur %8.2f  %s" % ((s - t0) / 1000.0, gap, (e - s) / 1000.0, name[:60]))
    prev_end = e
span = (rows[b][1] - t0) / 1000.0
print("step span %.2f us, kernels busy %.2f us, idle %.2f us" % (span, busy / 1000.0, span - busy / 1000.0))
