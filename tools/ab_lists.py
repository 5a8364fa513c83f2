#!/usr/bin/env python3
"""A/B timing of the C3 list kernels (bench.list_bench's workload: 100k entries, 1M lookups resident
in HBM): per setting, the mean of 20 mxp_list_check_device launches timed with HIP events, settings
alternated over 3 repetitions in one process.  Settings are environment assignments read per call
(e.g. MXP_LIST_IP_SPLIT=0); run once per library (MXP_LIB) to compare builds.
    python3 tools/ab_lists.py c3-ip "MXP_LIST_IP_SPLIT=1" "MXP_LIST_IP_SPLIT=0"
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from istio_amd import workloads as W  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402
import lists as L  # noqa: E402

kind, settings = sys.argv[1], sys.argv[2:] or [""]
if kind == "c3-ip":
    entries, syms = W.c3_ip_list(n_entries=100_000, n_lookups=1 << 20, seed=3)
    etype = L.IP_ADDRESSES
elif kind == "c3-str":
    entries, syms = W.c3_string_list(n_entries=100_000, n_lookups=1 << 20, seed=3)
    etype = L.CASE_INSENSITIVE_STRINGS
else:
    entries, syms = W.c3_regex_list(n_patterns=10_000, n_lookups=1 << 20, seed=3)
    etype = L.REGEX
eng = Engine(0)
lists = {}  # per setting: knobs read at list creation (MXP_LIST_RX16, MXP_LIST_LDS) take effect
for st in settings:
    for kv in st.split():
        k, v = kv.split("=", 1)
        os.environ[k] = v
    lists[st] = eng.list_create(etype, entries)
bs = [x.encode() for x in syms]
off = np.zeros(len(bs) + 1, dtype=np.uint64)
off[1:] = np.cumsum([len(b) for b in bs])
blob = np.frombuffer(b"".join(bs) + bytes(16), dtype=np.uint8)
d_blob = torch.from_numpy(blob.copy()).cuda()
d_off = torch.from_numpy(off.view(np.int64).copy()).cuda()
d_codes = torch.empty(len(bs), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
ref = None
res = {x: [] for x in settings}
for rep in range(3):
    for st in settings:
        for kv in st.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        lst = lists[st]
        for _ in range(3):
            lst.check_device(d_blob.data_ptr(), d_off.data_ptr(), len(bs), s.cuda_stream, d_codes.data_ptr())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record(s)
            lst.check_device(d_blob.data_ptr(), d_off.data_ptr(), len(bs), s.cuda_stream, d_codes.data_ptr())
            b.record(s)
        torch.cuda.synchronize()
        res[st].append(float(np.mean([a.elapsed_time(b) for a, b in ev])))
        codes = d_codes.cpu().numpy()
        if ref is None:
            ref = codes.copy()
        assert np.array_equal(codes, ref), "results differ between settings"
for st in settings:
    print("%-30s %s  ms per 1M lookups: %s" % (kind, st or "(default)", " ".join("%.4f" % x for x in res[st])))
print("lib", os.environ.get("MXP_LIB", "in-tree"), "codes identical across settings")
