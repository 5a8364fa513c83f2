#!/usr/bin/env python3
"""Summarise the two rocprofv3 --pmc passes of tools/pmc_session.sh.

Per kernel: mean FETCH_SIZE and WRITE_SIZE per dispatch (rocprofv3 reports KiB).  HBM bytes per
dispatch = 2 x FETCH_SIZE + WRITE_SIZE: on gfx950 FETCH_SIZE counts 128-byte memory-side reads at
64 bytes (MI355X_MICROARCH.md, HBM section).  Writes profiles/pmc_traffic.json (bytes per
evaluation = sum over the evaluation's kernels) and prints the table.

    python3 tools/pmc_summarize.py gpurun_out/pmc [--rules R --requests N]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (name prefixes: the per-slot-count instantiations, e.g. mxp_vtfill_imm5_kernel, included)
EVAL_KERNELS = ("mxp_fill_kernel", "mxp_fill_dtp_kernel", "mxp_vtfill", "mxp_vt_lookup_kernel",
                "mxp_vt_eval_kernel", "mxp_guard_kernel", "mxp_guard2_kernel", "mxp_eval_kernel", "mxp_index_kernel",
                "mxp_index_dtp_kernel", "mxp_index_dtp_lite_kernel", "mxp_index5_kernel", "mxp_dtp_sort_kernel", "mxp_dtp_apply_kernel",
                "mxp_inject_kernel", "mxp_hits_kernel", "mxp_hits_ragged_kernel", "mxp_hits_gate_kernel",
                "mxp_eval_deep_kernel", "mxp_quota", "mxp_dtp_hits_kernel",
                "mxp_list_kernel", "mxp_list_nfa_kernel", "mxp_list_rx_kernel", "mxp_list_rx_nfa_kernel",
                "mxp_list_ip_kernel", "mxp_list_str_kernel")


def per_kernel(path_glob, counter):
    vals = defaultdict(list)
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                vals[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--rules", type=int, default=10000)
    p.add_argument("--requests", type=int, default=1 << 20)
    p.add_argument("--workload", default="c2")
    p.add_argument("--list-entries", type=int, default=100_000)
    a, _ = p.parse_known_args()
    if a.workload.startswith("c3"):  # list workloads are keyed by their --list-entries (bench.list_bench)
        a.rules = a.list_entries
    # bench.py --workload c5 (C2 predicates + memquota in one step) looks its traffic up as "c2q"
    a.workload = {"c5": "c2q"}.get(a.workload, a.workload)
    fetch = per_kernel(os.path.join(a.dir, "FETCH_SIZE", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.dir, "WRITE_SIZE", "**", "*counter_collection.csv"), "WRITE_SIZE")
    table = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        table[k] = {"fetch_size_bytes": f, "write_size_bytes": w, "hbm_bytes": 2 * f + w}
        print("%-60s fetch %.4g B  write %.4g B  hbm(2F+W) %.4g B" % (k[:60], f, w, 2 * f + w))
    ev = {k: v for k, v in table.items() if any(k.startswith(e) for e in EVAL_KERNELS)}
    import sys
    sys.path.insert(0, ROOT)
    from bench import kernel_fingerprint
    out = {"workload": a.workload, "rules": a.rules, "requests": a.requests, "fingerprint": kernel_fingerprint(),
           "kernels": ev,
           "bytes_per_eval": sum(v["hbm_bytes"] for v in ev.values()) if ev else None,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE separate passes; hbm = 2*FETCH + WRITE (gfx950)"}
    json.dump(out, open(os.path.join(a.dir, "pmc_traffic_%s.json" % a.workload), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
