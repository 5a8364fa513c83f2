#!/usr/bin/env python3
"""The bench's end-to-end call alone (bench.end_to_end over a one-GPU group: narrow host shards ->
mxp_group_upload2 + mxp_group_resolve_uploaded), for rocprofv3 --kernel-trace --memory-copy-trace:
where the single call's time goes.  Prints the end_to_end block.
    python tools/e2e_group_prof.py [c2|c4] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    args = bench.parse(["--gen-procs", "1", "--fresh-steps", "1"])
    data = bench.Data(args, 1, {kind})
    manifest, rules = bench.rule_set(kind, args.rules)
    g = bench.make_group([0])
    g.set_vocabulary(manifest)
    assert (g.compile(rules) == 0).all()
    out = bench.end_to_end(g, [data.shards(kind, r) for r in range(3)], len(rules), reps)
    print(json.dumps({k: out[k] for k in ("ms_per_batch", "h2d_bytes_per_batch")}),
          json.dumps({"pipelined_ms": out["pipelined"]["ms_per_batch"]}))
    g.close()


if __name__ == "__main__":
    main()
