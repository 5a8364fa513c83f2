#!/usr/bin/env python3
"""The bench's fresh-batch loop alone (bench.fresh_batch_block over a one-GPU group), for rocprofv3
--kernel-trace --memory-copy-trace: where a fresh step's time goes (H2D copies, packer kernels,
evaluation).  Also prints the host time of each call of one step (upload, eval).
    python tools/fresh_group_prof.py [c2|c4] [steps] [narrow|wide]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wire = sys.argv[3] if len(sys.argv) > 3 else "narrow"
    args = bench.parse(["--gen-procs", "1", "--fresh-steps", str(steps)])
    data = bench.Data(args, 1, {kind})
    manifest, rules = bench.rule_set(kind, args.rules)
    g = bench.make_group([0])
    g.set_vocabulary(manifest)
    assert (g.compile(rules) == 0).all()
    out = bench.fresh_batch_block(g, [data.shards(kind, 1), data.shards(kind, 2)], steps, len(rules), wire)
    print({k: out[k] for k in ("ms_per_step", "upload_ms", "h2d_bytes_per_batch")})
    # one step's calls, timed on the host (after the loop: the sets are resident in pinned memory)
    sets, _, _keep = bench.host_sets([data.shards(kind, 1), data.shards(kind, 2)], wire)
    g.sync()
    t = [time.perf_counter()]
    a = bench.upload_set(g, sets[0], wire, True)
    t.append(time.perf_counter())
    b = bench.upload_set(g, sets[1], wire, True)
    t.append(time.perf_counter())
    g.eval(a)
    t.append(time.perf_counter())
    g.sync()
    t.append(time.perf_counter())
    g.eval(b)
    t.append(time.perf_counter())
    g.sync()
    t.append(time.perf_counter())
    d = [1e3 * (y - x) for x, y in zip(t, t[1:])]
    print("host ms: upload a %.3f, upload b %.3f, eval a call %.3f, eval a wait %.3f, eval b call %.3f, wait %.3f" % tuple(d))
    a.free()
    b.free()
    g.close()


if __name__ == "__main__":
    main()
