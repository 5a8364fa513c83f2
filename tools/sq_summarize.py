#!/usr/bin/env python3
"""LDS bank-conflict rate of the evaluation kernels from an SQ counter session (tools/sq_session.sh):
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per kernel (cycles stalled on bank conflicts per cycle the
LDS was busy with indexed accesses), plus the instruction mix.  Writes <dir>/sq_counters.json.
    python3 tools/sq_summarize.py gpurun_out/sq_c2 --workload c2"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

EVAL = ("mxp_fill_kernel", "mxp_fill_dtp_kernel", "mxp_vtfill", "mxp_guard_kernel", "mxp_guard2_kernel",
        "mxp_eval_kernel", "mxp_index_kernel", "mxp_index_dtp_kernel", "mxp_index_dtp_lite_kernel", "mxp_dtp_sort_kernel",
        "mxp_vt_lookup_kernel", "mxp_vt_eval_kernel", "mxp_inject_kernel", "mxp_dtp_hits_kernel", "mxp_quota",
        "mxp_list_kernel", "mxp_list_nfa_kernel", "mxp_list_rx_kernel", "mxp_list_rx_nfa_kernel",
        "mxp_list_ip_kernel", "mxp_list_str_kernel")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--workload", default="c2")
    a, _ = p.parse_known_args()
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "sq*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[row.get("Kernel_Name", "")][row["Counter_Name"]].append(float(row["Counter_Value"]))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_fingerprint
    out = {"workload": a.workload, "fingerprint": kernel_fingerprint(), "kernels": {},
           "method": "rocprofv3 --pmc SQ counters, 2 passes of 8; per-dispatch means; "
                     "bank_conflict_rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"}
    for k, cs in vals.items():
        if not k.startswith(EVAL):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        act = m.get("SQ_LDS_IDX_ACTIVE", 0.0)
        m["bank_conflict_rate"] = (m.get("SQ_LDS_BANK_CONFLICT", 0.0) / act) if act else 0.0
        out["kernels"][k.split("(")[0]] = m
    json.dump(out, open(os.path.join(a.dir, "sq_counters.json"), "w"), indent=1)
    print(json.dumps({k: round(v["bank_conflict_rate"], 4) for k, v in out["kernels"].items()}))


if __name__ == "__main__":
    main()
