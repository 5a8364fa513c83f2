"""The bench's fresh-batch loop alone (bench.fresh_batch_block: a new host batch uploaded and evaluated
every step), for rocprofv3 --hip-trace --kernel-trace --stats: where a fresh step's time goes (H2D
copies, allocations and frees, packer kernels, evaluation).  usage: fresh_prof.py c2|c4 [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from istio_amd.engine import Engine  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
manifest, rules, batch = bench.shard_workload(wl, 10000, 1 << 20, 0, 1)
batches = bench.fresh_batches(wl, 10000, 1 << 20, 0, 1)
eng = Engine(0)
eng.set_vocabulary(manifest)
eng.compile(rules)
R, N = len(rules), batch.n
dev = torch.device("cuda:0")
d_match = torch.empty(((R + 31) // 32, N), dtype=torch.int32, device=dev)
d_req_err = torch.empty(N, dtype=torch.uint8, device=dev)
hits = torch.zeros(R, dtype=torch.int64, device=dev)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)


def evaluate(db):
    db.eval_compact(d_match.data_ptr(), d_req_err.data_ptr(), hits.data_ptr(), stream.cuda_stream)


out = bench.fresh_batch_block(eng, batches, evaluate, steps, stream, R, 1)
print(wl, "fresh step ms %.3f upload ms %.3f" % (out["ms_per_step"], out["upload_ms"]))
