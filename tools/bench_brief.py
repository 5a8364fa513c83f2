#!/usr/bin/env python3
"""One-screen summary of a bench.py log: the headline and each block's step / kernel times."""
import json
import sys


def main(path):
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        print("C2 %.4f ms/step  %.4g pairs/s  frac %.3f" % (d["ms_per_step"], d["value"], d["roofline"]["frac"]))
        for k, v in d.items():
            if isinstance(v, dict) and "ms_per_step" in v and k not in ("fresh_batch",):
                print("%-6s %.4f ms/step kernel %s" % (k, v["ms_per_step"], v.get("kernel_ms")))
        for kk, vv in d.get("c3", {}).items():
            print("c3 %-5s %.4f ms/step kernel %.4f" % (kk, vv["ms_per_step"], vv["kernel_ms"]))
        for blk in ("fresh_batch", "fresh_batch_c4"):
            f = d.get(blk) or (d.get("c4") or {}).get(blk)
            if f:
                print("%s %.4f ms/step upload call %.4f ms, %d B/batch, frac %.3f" % (
                    blk, f["ms_per_step"], f["upload_ms"], f["h2d_bytes_per_batch"], f["roofline"]["frac"]))
        for blk, src in (("e2e", d), ("e2e_c4", d.get("c4") or {})):
            e = src.get("end_to_end")
            if e:
                print("%s %.4f ms single, %.4f ms pipelined" % (blk, e["ms_per_batch"], e["pipelined"]["ms_per_batch"]))
        cb = d.get("cpu_baseline")
        if cb:
            print("cpu %.4g %s" % (cb["value"], cb["unit"]))


if __name__ == "__main__":
    main(sys.argv[1])
