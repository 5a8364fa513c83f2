#!/usr/bin/env python3
"""Pipelined end-to-end Resolve: K engines on one GPU, each driven by its own host thread, each
resolving whole 1M-request batches (mxp_resolve_batch_ex, pinned batch and outputs) back to back.
One engine's upload (H2D) then overlaps another's action-list download (D2H) and host passes, as
a Check front end with several batch workers would run them.  Prints the per-batch throughput for
K = 1..--engines and checks every call's outputs against the first engine's.
    python3 tools/e2e_pipe.py [--workload c2|c4] [--engines 3] [--calls 6]"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c2")
    p.add_argument("--engines", type=int, default=3)
    p.add_argument("--calls", type=int, default=6, help="calls per engine in the timed region")
    p.add_argument("--requests", type=int, default=1 << 20)
    a = p.parse_args()
    import numpy as np
    import torch  # noqa: F401
    import bench
    from istio_amd.engine import Engine, pinned_batch
    manifest, rules, batch = bench.shard_workload(a.workload, 10000, a.requests, 0, 1)
    batch, arena = pinned_batch(batch)
    R = len(rules)
    engs = []
    for _ in range(a.engines):
        eng = Engine(0)
        eng.set_vocabulary(manifest)
        assert (eng.compile(rules) == 0).all()
        eng.set_resolver("destination.service", "istio-system", ["istio-system"] * R, np.ones(R, dtype=np.uint32),
                         np.zeros(R, dtype=np.uint8), np.zeros(R, dtype=np.uint8))
        engs.append(eng)
    st0, er0, off0, sel0 = (x.copy() for x in engs[0].resolve_arrays(batch, 0, ids16=True, pinned=True))
    cap = max(16, int(off0[-1]))
    for eng in engs[1:]:
        eng.resolve_arrays(batch, 0, cap, ids16=True, pinned=True)  # (warm: arenas, scratch)
    bad = []

    def worker(eng, calls, out, done):
        for _ in range(calls):
            st, er, off, sel = eng.resolve_arrays(batch, 0, cap, ids16=True, pinned=True)
        out.append(time.perf_counter())
        done.wait()  # (the last call's outputs checked after every worker's timed region)
        if not (np.array_equal(st, st0) and np.array_equal(er, er0) and np.array_equal(off, off0)
                and np.array_equal(sel, sel0)):
            bad.append(1)

    for k in range(1, a.engines + 1):
        ends = []
        done = threading.Barrier(k)
        ths = [threading.Thread(target=worker, args=(engs[i], a.calls, ends, done)) for i in range(k)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wall = max(ends) - t0  # (the workers' clocks stop before their checks)
        print("%s engines=%d: %d calls in %.2f ms -> %.3f ms per 1M-request batch (%.3e requests/s); "
              "action-list bytes per batch %d; outputs equal: %s" % (
                  a.workload, k, k * a.calls, wall * 1e3, wall * 1e3 / (k * a.calls), k * a.calls * batch.n / wall,
                  int(off0[-1]) * 2, not bad), flush=True)
    for eng in engs:
        eng.close()
    arena.free()


if __name__ == "__main__":
    main()
