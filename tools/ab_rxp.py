#!/usr/bin/env python3
"""Same-process A/B of the C3 regex-list kernels (1M lookups, 10k patterns): the union parts
(MXP_LIST_RXP=0, mxp_list_rx_kernel), literal-prefix dispatch (MXP_LIST_RXP=1) stepping tails from
global memory (mxp_list_rxp_kernel) or from a per-lane LDS copy (MXP_LIST_OPT bit 8,
mxp_list_rxp_lds_kernel), and two stage ablations of the global kernel (stop at the probe / at the
header: codes invalid; profiles/r6_s14_ab_rxp_stages.log); rounds alternated, HIP-event times,
codes compared.  (Round 6 also ran the union walk over lookups bucketed by their first three bytes,
an atomic counting sort first: the walk stayed at 0.089 ms and the sort cost 0.145 ms,
profiles/r6_s17_ab_rx_sorted.log, r6_s18_kernel_stats_ab_rx_sorted.csv -- removed.)  (Round 6 also
ran two lookups a lane with the tail walks stepped together: 0.176 against 0.126 ms,
profiles/r6_s15_ab_rxp_ilp.log -- removed.)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine, ListHandle  # noqa: E402


def main():
    pats, syms = W.c3_regex_list(n_patterns=10_000, n_lookups=1 << 20, seed=3)
    eng = Engine(0)
    lists = {}
    for name, rxp in (("union", "0"), ("rxp", "1")):
        os.environ["MXP_LIST_RXP"] = rxp
        lists[name] = eng.list_create(ListHandle.REGEX, pats)
    os.environ.pop("MXP_LIST_RXP")
    for name, lst in lists.items():
        print(name, "union parts / NFAs:", lst.regex_parts(), "dispatched patterns / prefixes:", lst.regex_dispatch())
    bs = [x.encode() for x in syms]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    blob = np.frombuffer(b"".join(bs) + bytes(16), dtype=np.uint8)
    d_blob = torch.from_numpy(blob.copy()).cuda()
    d_off = torch.from_numpy(off.view(np.int64).copy()).cuda()
    s = torch.cuda.Stream()
    variants = [("union", "union", "5"), ("rxp-global", "rxp", "5"), ("rxp-lds", "rxp", "13")]
    codes, times = {}, {v[0]: [] for v in variants}
    for rnd in range(6):
        for label, lst, opt in variants:
            os.environ["MXP_LIST_OPT"] = opt
            d_codes = torch.empty(len(bs), dtype=torch.int32, device="cuda")
            for _ in range(3):
                lists[lst].check_device(d_blob.data_ptr(), d_off.data_ptr(), len(bs), s.cuda_stream, d_codes.data_ptr())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                lists[lst].check_device(d_blob.data_ptr(), d_off.data_ptr(), len(bs), s.cuda_stream, d_codes.data_ptr())
            e1.record(s)
            torch.cuda.synchronize()
            times[label].append(e0.elapsed_time(e1) / 10)
            codes[label] = d_codes.cpu().numpy()
    for label in times:
        print("%-11s %s ms per 1M lookups (median %.4f)" % (label, " ".join("%.4f" % t for t in times[label]),
                                                             float(np.median(times[label]))))
    for label in codes:
        print(label, "codes equal to union:", bool(np.array_equal(codes[label], codes["union"])))


if __name__ == "__main__":
    main()
