#!/usr/bin/env python3
"""Phases of the end-to-end Resolve (mxp_resolve_batch on host bags, bench.end_to_end's call) with
MXP_TRACE=1, then the untraced call timed: C2 and C4 at 1M requests x 10k rules.
    python3 tools/e2e_trace.py [--workload c2|c4] [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c2")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--requests", type=int, default=1 << 20)
    p.add_argument("--pageable", action="store_true", help="the batch in pageable numpy memory (default: pinned)")
    p.add_argument("--u32", action="store_true", help="u32 rule ids (default: u16, mxp_resolve_batch_ex)")
    a = p.parse_args()
    import numpy as np
    import torch  # noqa: F401
    import bench
    from istio_amd.engine import Engine, pinned_batch
    manifest, rules, batch = bench.shard_workload(a.workload, 10000, a.requests, 0, 1)
    if not a.pageable:
        batch, arena = pinned_batch(batch)
    ids16 = not a.u32
    R = len(rules)
    for traced in (True, False):
        os.environ["MXP_TRACE"] = "1" if traced else "0"
        eng = Engine(0)
        eng.set_vocabulary(manifest)
        assert (eng.compile(rules) == 0).all()
        eng.set_resolver("destination.service", "istio-system", ["istio-system"] * R, np.ones(R, dtype=np.uint32),
                         np.zeros(R, dtype=np.uint8), np.zeros(R, dtype=np.uint8))
        status, _, off, _ = eng.resolve_arrays(batch, 0, ids16=ids16, pinned=not a.pageable)
        cap = max(16, int(off[-1]))
        ts = []
        for k in range(a.reps):
            if traced:
                print("-- traced call %d" % k, file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            status, _, off, sel = eng.resolve_arrays(batch, 0, cap, ids16=ids16, pinned=not a.pageable)
            ts.append(time.perf_counter() - t0)
        print("%s %s %s %s: ms per call %s (median %.2f); selected/request %.1f, error requests %d" % (
            a.workload, "pageable" if a.pageable else "pinned", "u32" if a.u32 else "u16",
            "traced" if traced else "untraced", ["%.2f" % (t * 1e3) for t in ts],
            float(np.median(ts)) * 1e3, float(off[-1]) / batch.n, int((status == 3).sum())), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
