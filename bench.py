#!/usr/bin/env python3
"""Benchmark: request x rule predicate evaluations per second (BASELINE.json `metric`).

Headline workload (per GPU): the C2 rule family of BASELINE.json configs[1] (`destination.service ==
... && request.path.startsWith(...) && source.ip != ip(...)`) scaled to the metric's 10k rules, over
1M synthetic requests (Zipf(1.1) services) resident in HBM -- the per-GPU shard of configs[4]
(8 x MI355X, 8M requests).  A step = one evaluation of every rule against every request of the
shard (the full predicate bitmap) + the per-rule hit counters, reduced over RCCL when N > 1 with one
all-reduce per step (istio_amd.dist.StepCounters).

The default run also measures C4 (configs[3]: 10k Pilot-style route rules x 1M requests) with the
same step structure and reports it as the extra "c4" block of the same JSON line (--no-c4: skip),
and C3 (configs[2]: CIDR, case-insensitive string and regex lists, 100k entries x 1M lookups) as
the "c3" block (--no-c3: skip).  Each predicate block also carries a "fresh_batch" figure: a new
1M-request batch uploaded from host memory and evaluated every step (PCIe-inclusive).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rules R] [--requests N_PER_GPU]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
    python bench.py --workload c4 | c5 | c3-ip | c3-str | c3-regex | c5-quota

With N GPUs every rank evaluates its contiguous shard (istio_amd.dist.shard_bounds) of ONE seeded
batch of N x --requests requests (configs[4]: 8 x 1M).  The default line also carries a "c5" block:
the C2 predicates + the shard's memquota batch + one all-reduce of hits[R] ++ quota_delta[K].

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
QUOTA_KEYS = 1024


def host_threads():
    """CPU threads for the host baselines: every CPU the process may use (os.cpu_count(), bounded by
    its affinity set and by OMP_NUM_THREADS when the environment sets it -- the GPU box reports the
    whole machine's CPUs but grants a share of 16)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    if os.environ.get("OMP_NUM_THREADS"):
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    return max(1, n)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rules", type=int, default=10000)
    p.add_argument("--requests", type=int, default=1 << 20)
    p.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    p.add_argument("--cpu-threads", type=int, default=host_threads())
    p.add_argument("--list-cpu-seconds", type=float, default=4.0, help="CPU-baseline sample per C3 list kind")
    p.add_argument("--no-c3", action="store_true", help="default run: skip the extra C3 list block")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--quota-serial", action="store_true",
                   help="C5: the memquota batch after the evaluation on one stream (default: a second stream beside it)")
    p.add_argument("--no-c4", action="store_true", help="default run: skip the extra C4 block")
    p.add_argument("--no-c5", action="store_true", help="default run: skip the extra C5 block")
    p.add_argument("--workload", default="c2", choices=["c2", "c4", "c5", "c3-ip", "c3-str", "c3-regex", "c5-quota"],
                   help="c2 (default, the BASELINE metric; + a C4 block); c4 route rules; c5 = C2 predicates + "
                        "memquota with one combined all-reduce; C3 lists; c5-quota memquota alone")
    p.add_argument("--list-entries", type=int, default=100_000)
    p.add_argument("--e2e-reps", type=int, default=3, help="end-to-end resolve calls timed (median); 0 skips the end-to-end block (profiling sessions)")
    p.add_argument("--fresh-steps", type=int, default=10,
                   help="steps of the fresh-batch block (upload + evaluation of a new 1M batch per step); 0 skips it")
    p.add_argument("--error-output", default="compact", choices=["compact", "bitmap"],
                   help="compact: per-request error flags (a Resolve's view); bitmap: the full error bitmap")
    return p.parse_args()


def cpu_baseline(manifest, rules, batch, seconds, threads, chunk=256):
    """The oracle (C restatement of the reference interpreter, oracle/il_interp.c, with the C
    restatement of Go's regexp for `matches`) on host cores, time-bounded sample of the same workload.

    Main figure: rules precompiled -- the reference's best case, its expression cache holding every
    rule (--expressionEvalCacheSize >= R) -- while `matches` compiles its pattern on every call, as
    regexp.MatchString does (externs.go:118-120).  "lru1024": the reference's default cache of 1024
    expressions (mixer/pkg/il/evaluator/evaluator.go:157-182) with R = 10k rules evaluated in turn
    misses on every call, so every pair also pays expr.Parse + EvalType + compiler.Compile; that
    compile cost is measured on the C++ restatement of the front end and compiler (a host-only
    engine compiling the rules one at a time) and added per pair."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ev = oracle.OracleEvaluator(manifest)
    oracle.regex_cache(False)  # regexp.MatchString compiles the pattern on every call
    oracle.oracle_matrix(ev, rules, batch, 0, 1, threads=1)  # compile all rules (untimed)
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done + chunk <= batch.n:
        oracle.oracle_matrix(ev, rules, batch, done, done + chunk, threads=threads)
        done += chunk
    dt = time.perf_counter() - t0
    oracle.regex_cache(True)
    pairs = done * len(rules)
    rate = pairs / dt
    # compile cost per rule (single thread), on a sample of the rules
    from istio_amd.engine import Engine
    eng = Engine(-1)
    eng.set_vocabulary(manifest)
    sample = rules[:: max(1, len(rules) // 300)]
    t1 = time.perf_counter()
    for r in sample:
        eng.compile([r])
    t_compile = (time.perf_counter() - t1) / len(sample)
    t_pair = threads / rate  # one thread's seconds per pair
    lru = {"value": threads / (t_pair + t_compile), "unit": "pairs/s", "cores": threads,
           "compile_us_per_rule": t_compile * 1e6,
           "variant": "expressionEvalCacheSize=1024 (default) with R=%d rules: every EvalPredicate recompiles" % len(rules)}
    return {"value": rate, "unit": "pairs/s", "cores": threads, "host_cpus": os.cpu_count(), "kind": "port",
            "sample": "%d requests x %d rules (%.1fs, oracle C restatement, rules precompiled, regexps compiled "
                      "per matches call)" % (done, len(rules), dt),
            "lru1024": lru}


def kernel_fingerprint():
    """sha1 of the engine's kernel and launch sources: a PMC profile is valid for this build only."""
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(ROOT, "istio_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")) or f in ("engine.cpp", "pack_device.cpp", "lower.cpp", "vmopt.cpp"):
            h.update(f.encode())
            h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()


def measured_traffic(workload, rules, requests):
    """HBM bytes per evaluation from the committed PMC profile of THIS build (tools/pmc_summarize.py:
    FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, FETCH doubled for gfx950; the profile
    records kernel_fingerprint() of the sources it measured), when one exists for this workload
    size; else None -- a profile of other kernels is not reported."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % workload)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if (d.get("workload") == workload and d.get("rules") == rules and d.get("requests") == requests
            and d.get("fingerprint") == kernel_fingerprint()):
        return d.get("bytes_per_eval")
    return None


def lds_conflicts(workload):
    """LDS bank-conflict rate per evaluation kernel from the committed SQ counter session of THIS
    build and workload (tools/sq_session.sh + tools/sq_summarize.py ->
    profiles/sq_counters_<workload>.json, keyed by kernel_fingerprint()), or None."""
    path = os.path.join(ROOT, "profiles", "sq_counters_%s.json" % workload)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("workload") != workload or d.get("fingerprint") != kernel_fingerprint():
        return None
    return {k: {"bank_conflict_cycles": v.get("SQ_LDS_BANK_CONFLICT"), "lds_active_cycles": v.get("SQ_LDS_IDX_ACTIVE"),
                "rate": v.get("bank_conflict_rate")} for k, v in d.get("kernels", {}).items()}


LAST_ENQUEUE_MS = None


class StepEvent:
    """A HIP timing event recorded without the system-scope fence (hipEventDisableSystemFence): the
    per-step events of the timed region.  A default event's record (torch.cuda.Event) writes back
    and invalidates the caches for host visibility, and the next step's first kernel waits that out:
    ~14 us of every ~0.4 ms C2 step.  These events only time the stream's work; the region itself
    is still bracketed by synchronize().  Same HIP runtime as torch's (libamdhip64.so.7, already
    loaded by `import torch`)."""
    _hip = None

    def __init__(self):
        import ctypes
        if StepEvent._hip is None:
            import torch  # noqa: F401  (its runtime first: one HIP runtime per process)
            h = ctypes.CDLL("libamdhip64.so.7")
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            StepEvent._hip = h
        self._ct = ctypes
        self.ev = ctypes.c_void_p()
        if StepEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.ev), 0x20000000):  # hipEventDisableSystemFence
            raise RuntimeError("hipEventCreateWithFlags failed")

    def wait(self, stream):
        """`stream` waits for this event's record (hipStreamWaitEvent: an ordering, no host wait)."""
        h = StepEvent._hip
        h.hipStreamWaitEvent.argtypes = [self._ct.c_void_p, self._ct.c_void_p, self._ct.c_uint]
        if h.hipStreamWaitEvent(self._ct.c_void_p(stream.cuda_stream), self.ev, 0):
            raise RuntimeError("hipStreamWaitEvent failed")

    def record(self, stream=None):
        if StepEvent._hip.hipEventRecord(self.ev, self._ct.c_void_p(stream.cuda_stream if stream is not None else None)):
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end):
        ms = self._ct.c_float()
        if StepEvent._hip.hipEventElapsedTime(self._ct.byref(ms), self.ev, end.ev):
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def __del__(self):
        if StepEvent._hip is not None and self.ev:
            StepEvent._hip.hipEventDestroy(self.ev)


def timed_loop(step, steps, warmup, world, stream):
    """W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize; returns the
    slowest rank's seconds and the per-step HIP-event durations (ms) recorded on `stream`.  (Without
    a GPU -- the gloo CPU tests of the step -- there is nothing to synchronise and no events.)"""
    import torch
    import torch.distributed as dist
    from istio_amd import dist as D
    gpu = torch.cuda.is_available()
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    # (BENCH_FENCED_EVENTS=1: torch's default events instead, for same-box A/B of the fence's cost)
    mk = (lambda: torch.cuda.Event(enable_timing=True)) if os.environ.get("BENCH_FENCED_EVENTS") else StepEvent
    evs = [(mk(), mk()) if gpu else (None, None) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(*evs[k])
    global LAST_ENQUEUE_MS  # host time to enqueue one step (the GPU idles between steps if >= its time)
    LAST_ENQUEUE_MS = (time.perf_counter() - t0) / max(steps, 1) * 1e3
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = [a.elapsed_time(b) for a, b in evs] if gpu else []
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else None
    return D.max_over_ranks(elapsed, dev), ev_ms


PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 host link, spec (MI355X_MICROARCH.md)


def batch_h2d_bytes(batch):
    """Bytes of the host columnar batch mxp_batch_upload copies to the device (Go-owned bags)."""
    n = sum(k.nbytes for k in batch.kinds) + sum(v.nbytes for v in batch.values)
    return int(n + batch.str_blob.nbytes + batch.str_offsets.nbytes + batch.time_sec.nbytes + batch.time_nsec.nbytes
               + batch.map_offsets.nbytes + batch.map_keys.nbytes + batch.map_values.nbytes)


def fresh_batches(kind, n_rules, requests_per_gpu, rank, world):
    """Two further 1M-request batches of the same seeded stream (the shards after this rank's own,
    as if two more batches of configs[4] arrived): the fresh-batch block alternates them."""
    from istio_amd import dist as D
    from istio_amd import workloads as W
    n_total = requests_per_gpu * world
    out = []
    for k in (1, 2):
        lo, hi = D.shard_bounds(n_total, rank, world)
        shard = (lo + k * n_total, hi + k * n_total)
        if kind == "c4":
            out.append(W.c4_workload(n_rules=n_rules, n_requests=3 * n_total, seed=4, shard=shard)[2])
        else:
            out.append(W.c2_workload(n_rules=n_rules, n_requests=3 * n_total, seed=2, shard=shard)[2])
    return out


def fresh_batch_block(eng, batches, evaluate, steps, stream, n_rules, world):
    """Every step takes a NEW batch from host memory, double-buffered: mxp_batch_upload_ex of batch
    k + 1 with MXP_UPLOAD_NO_WAIT (its H2D copies queued and the batch checked; the device packer --
    interning, gather, pre-tables, value-class counts -- runs after them), then the evaluation of
    batch k (its first evaluation finishes its packing: class tables, string heads, dictionary;
    enqueued); a host batch is refilled only after mxp_batch_wait_copied of its previous upload, two
    steps back.  Batch k + 1's copies queue behind batch k's on the copy stream, so the link stays
    busy while the host works on the previous batch and the device packs and evaluates.  The two
    host batches alternate; a device batch is freed three steps after its evaluation.  PCIe-inclusive.
    The host batches live in pinned memory (mxp_host_alloc), as a binding's reused packing arenas do
    (INTEGRATION.md 2e): their copies are DMA at the link's rate."""
    import numpy as np
    import torch
    from istio_amd.engine import pinned_batch
    pinned = [pinned_batch(b) for b in batches]
    batches = [b for b, _ in pinned]
    keep, up_s, pending, copying = [], [], [], []
    h2d = [batch_h2d_bytes(b) for b in batches]

    def one(k):
        if len(copying) >= len(batches):  # (this step's host batch was uploaded len(batches) steps ago)
            copying.pop(0).wait_copied()
        t0 = time.perf_counter()
        db = eng.upload(batches[k % len(batches)], no_wait=True)  # (copies queued, batch checked)
        up_s.append(time.perf_counter() - t0)
        copying.append(db)
        if pending:  # (the previous batch, uploaded one step ago)
            prev = pending.pop()
            evaluate(prev)
            keep.append(prev)
            if len(keep) > 3:
                keep.pop(0).free()
        pending.append(db)
    for k in range(3):  # warm-up (allocations)
        one(k)
    torch.cuda.synchronize()
    up_s.clear()
    t0 = time.perf_counter()
    for k in range(steps):  # (k uploads and k evaluations)
        one(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    while pending:
        evaluate(pending[0])
        keep.append(pending.pop())
    torch.cuda.synchronize()
    copying.clear()
    while keep:
        keep.pop(0).free()
    N = batches[0].n
    up = float(np.mean(up_s))
    bytes_step = float(np.mean([h2d[k % len(batches)] for k in range(steps)]))
    return {"ms_per_step": dt * 1e3, "upload_ms": up * 1e3, "requests_per_s": world * N / dt,
            "pairs_per_s": world * N * n_rules / dt, "steps": steps, "h2d_bytes_per_batch": int(bytes_step),
            "roofline": {"bound": "pcie", "achieved": bytes_step / dt / 1e9, "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                         "frac": bytes_step / dt / 1e9 / PCIE_PEAK_GBS, "traffic": None,
                         "kernel": "mxp_batch_upload: H2D copy of the host columnar batch + the device packer "
                                   "(intern, gather, pool, pre-tables, value-class dictionary, heads); "
                                   "achieved = batch bytes / step wall time (upload + evaluation, pipelined)"},
            "upload_call_gbs": bytes_step / up / 1e9,
            "host_memory": "pinned (mxp_host_alloc arenas)",
            "path": "host columnar batch (a new 1M-request batch every step) -> mxp_batch_upload (batch k + 1) -> "
                    "evaluation (batch k: compact errors, fused hit counters); wall time per step, PCIe-inclusive"}


def shard_workload(kind, n_rules, requests_per_gpu, rank, world):
    """This rank's shard of ONE seeded batch of requests_per_gpu x world requests (configs[4]: the
    8 x 1M batch), contiguous per rank (dist.shard_bounds); the rule set is the same on every rank."""
    from istio_amd import dist as D
    from istio_amd import workloads as W
    n_total = requests_per_gpu * world
    shard = D.shard_bounds(n_total, rank, world)
    if kind == "c4":
        return W.c4_workload(n_rules=n_rules, n_requests=n_total, seed=4, shard=shard)
    manifest, _, batch = W.c2_workload(n_rules=n_rules, n_requests=n_total, seed=2, shard=shard)
    return manifest, W.c2_rules(n_rules, seed=2)[0], batch


def make_step(ctr, evaluate, quota_alloc=None, stream=None, qstream=None):
    """The bench step: evaluate every pair of the shard with the hit counters
    accumulated into the step's hits view, optionally the shard's memquota batch with its per-key
    deltas into the quota view, then the step's ONE all-reduce of hits[R] ++ quota_delta[K]
    (StepCounters.end_step; nothing on a single process).  ev0 / ev1 bracket the kernels.
    With `qstream` the memquota batch runs on that second stream beside the evaluation (the two
    touch disjoint buffers; its latency-bound replay overlaps the predicate kernels), forked after
    the counters are zeroed and joined before the all-reduce."""
    fork = join = None
    if qstream is not None:  # (ordering events without the system-scope fence: StepEvent)
        fork, join = StepEvent(), StepEvent()

    def step(ev0=None, ev1=None):
        ctr.begin_step()
        views = ctr.views()
        if ev0 is not None:
            ev0.record(stream)
        if quota_alloc is not None and qstream is not None:
            fork.record(stream)
            fork.wait(qstream)
            quota_alloc(views[1], qstream.cuda_stream)
            join.record(qstream)
        evaluate(views[0])
        if quota_alloc is not None:
            if qstream is not None:
                join.wait(stream)
            else:
                quota_alloc(views[1], stream.cuda_stream if stream is not None else None)
        if ev1 is not None:
            ev1.record(stream)
        ctr.end_step()
    return step


def list_bench(args, rank, world, local, kind=None, emit=True):
    """C3 (BASELINE configs[2]): 100k-entry CIDR / string / regex lists, 1M lookups per GPU resident
    in HBM; one step = HandleListEntry for every lookup (mxp_list_check_device, one kernel).
    Returns the result dict (printed as the line when emit)."""
    import numpy as np
    import torch
    from istio_amd import workloads as W
    from istio_amd.engine import Engine
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lists as L
    kind = kind or args.workload
    n_look = args.requests
    if kind == "c3-ip":
        entries, syms = W.c3_ip_list(n_entries=args.list_entries, n_lookups=n_look, seed=3 + 1000 * rank)
        etype = L.IP_ADDRESSES
    elif kind == "c3-str":
        entries, syms = W.c3_string_list(n_entries=args.list_entries, n_lookups=n_look, seed=3 + 1000 * rank)
        etype = L.CASE_INSENSITIVE_STRINGS
    else:
        entries, syms = W.c3_regex_list(n_patterns=min(args.list_entries, 10_000), n_lookups=n_look,
                                        seed=3 + 1000 * rank)
        etype = L.REGEX
    eng = Engine(local)
    t0 = time.perf_counter()
    lst = eng.list_create(etype, entries)
    t_compile = time.perf_counter() - t0
    bs = [x.encode() for x in syms]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    blob = np.frombuffer(b"".join(bs) + bytes(16), dtype=np.uint8)
    dev = torch.device("cuda", local)
    d_blob = torch.from_numpy(blob.copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    d_codes = torch.empty(len(bs), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step(e0=None, e1=None):
        if e0 is not None:
            e0.record(stream)
        lst.check_device(d_blob.data_ptr(), d_off.data_ptr(), len(bs), stream.cuda_stream, d_codes.data_ptr())
        if e1 is not None:
            e1.record(stream)
    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, world, stream)
    kernel_ms = float(np.mean(ev_ms))
    n = len(bs)
    alg = int(off[-1]) + 8 * (n + 1) + 4 * n  # symbol bytes + offsets read, one code written each
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    # the kernel the step launches (lists.cpp mxp_list_check_device): CIDR lookups regrouped by
    # address family, string lookups by the register window, regex lists with their automata staged
    # in LDS unless MXP_LIST_LDS=0
    kname = {"c3-ip": "mxp_list_ip_kernel", "c3-str": "mxp_list_str_kernel"}.get(
        kind, "mxp_list_rx_kernel" if os.environ.get("MXP_LIST_LDS", "1") != "0" else "mxp_list_kernel")
    out = {"metric": "list-adapter lookups/sec (%s, %d entries)" % (kind, lst.num_entries()),
           "value": world * n * args.steps / elapsed, "unit": "lookups/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (seeded C3 %s list and lookups; symbols resident in HBM)" % kind[3:],
           "config": {"workload": "C3 %s list, %d entries, %d lookups per GPU (configs[2])" % (kind[3:], len(entries), n),
                      "entries": len(entries), "lookups_per_gpu": n, "parallelism": "lookup-sharded dp%d" % world},
           "kernel_ms": kernel_ms, "list_compile_s": t_compile,
           "lds_bank_conflicts": lds_conflicts(kind),
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": measured_traffic(kind, args.list_entries, n),
                        "kernel": kname, "alg_bytes_per_launch": alg}}
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = list_cpu_baseline(L, kind, entries, syms, args.list_cpu_seconds, args.cpu_threads)
    del d_blob, d_off, d_codes, lst
    if rank == 0 and emit:
        print(json.dumps(out))
    return out


def quota_setup(eng, n_requests, rank, world, dev):
    """memquota state for QUOTA_KEYS keys and this rank's quota requests: the global arrival stream
    routed by key owner (workloads.quota_workload, dist.key_owners: LPT over the keys' expected
    frequencies), resident in HBM."""
    import numpy as np
    import torch
    from istio_amd import workloads as W
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=QUOTA_KEYS, n_requests=n_requests, seed=5, rank=rank,
                                                 world=world)
    q = eng.quota_create(mx, vd)
    dk = torch.from_numpy(keys.view(np.int32).copy()).to(dev)
    da = torch.from_numpy(amounts.copy()).to(dev)
    db = torch.from_numpy(be.copy()).to(dev)
    dg = torch.empty(len(keys), dtype=torch.int64, device=dev)
    return (mx, vd, keys, amounts, be), q, (dk, da, db, dg)


def quota_bench(args, rank, world, local):
    """C5 memquota (BASELINE configs[4]): K = 1024 quota keys, each owned by one rank (dist.key_owners), the
    quota requests routed to their key's owner in arrival order (~1M per GPU); a step = batched
    HandleQuota (sort by key + per-key replay) and, when N > 1, the all-reduce of the per-key deltas."""
    import numpy as np
    import torch
    from istio_amd import dist as D
    from istio_amd.engine import Engine
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import memquota as M
    eng = Engine(local)
    dev = torch.device("cuda", local)
    (mx, vd, keys, amounts, be), q, (dk, da, db, dg) = quota_setup(eng, args.requests, rank, world, dev)
    ctr = D.StepCounters([QUOTA_KEYS], dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    now = [1_500_000_000 * 10**9]

    def step(e0=None, e1=None):
        ctr.begin_step()
        (delta,) = ctr.views()
        if e0 is not None:
            e0.record(stream)
        q.alloc_device(len(keys), dk.data_ptr(), da.data_ptr(), db.data_ptr(), now[0], stream.cuda_stream,
                       dg.data_ptr(), delta.data_ptr())
        if e1 is not None:
            e1.record(stream)
        ctr.end_step()
        now[0] += 10**8
    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, world, stream)
    kernel_ms = float(np.mean(ev_ms))
    n = len(keys)
    n_all = int(D.sum_over_ranks(float(n)))  # quota requests of all ranks (routing by key owner)
    alg = n * (4 + 8 + 1 + 8)  # key, amount, best effort read; granted written
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    out = {"metric": "memquota HandleQuota requests/sec (%d keys)" % QUOTA_KEYS,
           "value": n_all * args.steps / elapsed,
           "unit": "requests/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "int64", "data": "synthetic (seeded C5 quota requests routed by key owner; resident in HBM)",
           "config": {"workload": "C5 memquota, %d keys, %d requests per GPU (configs[4])" % (QUOTA_KEYS, n),
                      "keys": QUOTA_KEYS, "requests_per_gpu": n, "parallelism": "key-owner-sharded dp%d" % world},
           "kernel_ms": kernel_ms,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                        "kernel": "counting sort by key (mxp_quota_hist / binscan / scatter) + mxp_quota_kernel",
                        "alg_bytes_per_launch": alg}}
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        # the C restatement (oracle/memquota_oracle.c): the same batches, keys in parallel on the
        # host's cores (each key's requests sequential, as the reference's mutex runs them)
        ref = M.CMemquota(mx, vd)
        t0 = time.perf_counter()
        done, t_ns = 0, 1_500_000_000 * 10**9
        while done == 0 or (time.perf_counter() - t0 < args.cpu_sample_seconds and done < 64 * n):
            ref.handle_batch(keys, amounts, be, t_ns, threads=args.cpu_threads)
            done += n
            t_ns += 10**8
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": done / dt, "unit": "requests/s", "cores": args.cpu_threads,
                               "host_cpus": os.cpu_count(), "kind": "port",
                               "sample": "%d requests (%d batches of %d, %.1fs), memquota C restatement, keys in "
                                         "parallel on %d threads" % (done, done // n, n, dt, args.cpu_threads)}
    if rank == 0:
        print(json.dumps(out))


def list_cpu_baseline(L, kind, entries, syms, seconds, threads):
    """The list restatements timed on host cores, compiled and multi-threaded (OpenMP over the
    lookups): the IP list is the reference's linear IPNet scan (ipList.go:77-92); case-insensitive
    strings a hash set after Go's strings.ToUpper (stringList.go:51-80, a Go map); regexes the Go
    regexp restatement, patterns tried in order until one matches (regexList.go:26-33)."""
    if kind == "c3-ip":
        ref = L.IPList(entries)
    elif kind == "c3-str":
        ref = L.CStringList(entries, case_insensitive=True)
    else:
        ref = L.RegexList(entries)
    # (chunks of >= 4096 lookups: the regex restatement compiles its patterns once per call, a few
    # percent of a chunk's time)
    chunk, done = 4096, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done + chunk <= len(syms):
        ref.found(syms[done:done + chunk], threads=threads)
        done += chunk
        chunk = min(chunk * 2, 1 << 18)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "lookups/s", "cores": threads, "host_cpus": os.cpu_count(),
            "kind": "port",
            "sample": "%d lookups (%.1fs) against all %d entries, oracle C restatement on %d threads" % (
                done, dt, len(entries), threads)}


def end_to_end(eng, batch, n_rules, reps):
    """The whole Check-path call from Go-owned bags to action lists: the host
    columnar batch -> mxp_resolve_batch (device packing and interning, evaluation of every pair,
    per-request resolution and action-list gather on the device) -> status / first-error rule /
    selected rules back in host memory.  Every rule sits in the default namespace with one variety,
    so each request's action list is every rule whose predicate holds (resolver.go:202-238).
    PCIe-inclusive; not `value` (whose inputs are resident in HBM)."""
    import numpy as np
    from istio_amd.engine import pinned_batch
    eng.set_resolver("destination.service", "istio-system", ["istio-system"] * n_rules,
                     np.ones(n_rules, dtype=np.uint32), np.zeros(n_rules, dtype=np.uint8),
                     np.zeros(n_rules, dtype=np.uint8))
    batch, arena = pinned_batch(batch)  # (the binding's packing arena: pinned host memory)
    ids16 = n_rules <= 65536  # mxp_resolve_batch_ex(MXP_RESOLVE_IDS_U16)
    status, _, off, _ = eng.resolve_arrays(batch, 0, ids16=ids16, pinned=True)  # warm-up (allocations)
    cap = max(16, int(off[-1]))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        status, _, off, _ = eng.resolve_arrays(batch, 0, cap, ids16=ids16, pinned=True)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    sel_bytes = int(off[-1]) * (2 if ids16 else 4)
    return {"pairs_per_s": batch.n * n_rules / t, "requests_per_s": batch.n / t, "ms_per_batch": t * 1e3,
            "reps": reps, "selected_per_request": float(off[-1]) / max(batch.n, 1),
            "pred_error_requests": int((status == 3).sum()), "rule_ids": "u16" if ids16 else "u32",
            "action_list_bytes": sel_bytes, "action_list_ms_at_50GBps": sel_bytes / 50e9 * 1e3,
            "x_action_list_at_50GBps": t * 1e3 / max(sel_bytes / 50e9 * 1e3, 1e-9),
            "host_memory": "pinned batch and outputs (mxp_host_alloc arenas)",
            "path": "host columnar bags -> mxp_resolve_batch_ex (device pack + namespaces + compact evaluation + "
                    "first errors from the records + device scan + action-list gather) -> host action lists; median "
                    "of reps, PCIe-inclusive"}


def predicate_bench(args, kind, rank, world, local, with_quota=False):
    """One predicate workload (c2 / c4) on this rank's 1M-request shard; returns the result dict.

    Step: evaluate every (request, rule) pair with the per-rule hit counters fused into the
    evaluation kernels (accumulated into the step's counter buffer), optionally the memquota
    HandleQuota batch of the rank's quota requests (per-key deltas into the same buffer), then ONE
    all-reduce of hits[R] ++ quota_delta[K] when N > 1."""
    import numpy as np
    import torch
    from istio_amd import dist as D
    from istio_amd import workloads as W
    from istio_amd.engine import Engine

    dev = torch.device("cuda", local)
    # ONE seeded batch of requests_per_gpu x N requests (configs[4]: 8 x 1M), each rank evaluating
    # its contiguous shard (dist.shard_bounds) against the replicated rule set
    manifest, rules, batch = shard_workload(kind, args.rules, args.requests, rank, world)
    if kind == "c4":
        metric, workload = ("request x rule predicate evals/sec at 10k rules (C4 route rules)",
                            "C4 Pilot-style route rules R=%d, %d requests per GPU (configs[3])")
    else:
        metric, workload = ("request x rule predicate evals/sec at 10k rules",
                            "C2 rules scaled to R=%d, %d requests per GPU (configs[1] family, configs[4] shard)")
        if with_quota:
            workload = "C5: C2 rules R=%d, %d requests per GPU + memquota (configs[4])"
    eng = Engine(local)
    eng.set_vocabulary(manifest)
    st = eng.compile(rules)
    assert (st == 0).all()
    t_pack = time.perf_counter()
    db = eng.upload(batch)
    t_pack = time.perf_counter() - t_pack

    R, N = len(rules), batch.n
    Wd = (R + 31) // 32
    d_match = torch.empty((Wd, N), dtype=torch.int32, device=dev)
    # error output: per-request error flags (compact, default; what a Resolve needs) or the full
    # error bitmap (--error-output bitmap; the parity tests' reference form)
    compact = args.error_output == "compact"
    d_err = torch.empty((Wd, N) if not compact else (1,), dtype=torch.int32, device=dev)
    d_req_err = torch.empty(N if compact else 1, dtype=torch.uint8, device=dev)

    def evaluate(hits_ptr):
        if compact:
            db.eval_compact(d_match.data_ptr(), d_req_err.data_ptr(), hits_ptr, sh)
        elif hits_ptr:
            db.eval_hits(d_match.data_ptr(), d_err.data_ptr(), hits_ptr, sh)
        else:
            db.eval(d_match.data_ptr(), d_err.data_ptr(), sh)
    # a real (non-null) HIP stream shared by libmxp, events and RCCL.  C5's memquota stream runs at the
    # higher priority: its latency-bound replay is dispatched ahead of the fill's workgroups (C5 0.5226
    # -> 0.5186 ms per step alternated, profiles/r4_s30_c5_*.log; BENCH_STREAM_PRIO / BENCH_QSTREAM_PRIO
    # override, a lower number is a higher priority)
    stream = torch.cuda.Stream(dev, priority=int(os.environ.get("BENCH_STREAM_PRIO", "0")))
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    quota = None
    if with_quota:
        quota = quota_setup(eng, N, rank, world, dev)
    ctr = D.StepCounters([R] + ([QUOTA_KEYS] if quota else []), dev)
    now = [1_500_000_000 * 10**9]

    def quota_alloc(delta, qsh):
        (_, q, (dk, da, dbe, dg)) = quota
        q.alloc_device(dk.numel(), dk.data_ptr(), da.data_ptr(), dbe.data_ptr(), now[0], qsh, dg.data_ptr(),
                       delta.data_ptr())
        now[0] += 10**8
    qstream = (torch.cuda.Stream(dev, priority=int(os.environ.get("BENCH_QSTREAM_PRIO", "-1")))
               if quota is not None and not args.quota_serial else None)
    step = make_step(ctr, lambda hits: evaluate(hits.data_ptr()), quota_alloc if quota is not None else None, stream,
                     qstream)

    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, world, stream)
    step_kernel_ms = float(np.mean(ev_ms))
    value = world * N * R * args.steps / elapsed

    # per-kernel durations (HIP events recorded by libmxp around each launch, on `stream`), in a
    # separate pass so the timed region above carries no extra synchronisation; the evaluation as
    # the step runs it, hit counters included (the span ends after the counters)
    scratch_hits = torch.zeros(R, dtype=torch.int64, device=dev)
    eng.set_timing(True)
    per = []
    for _ in range(args.steps):
        evaluate(scratch_hits.data_ptr())
        per.append(eng.kernel_times(3))
    eng.set_timing(False)
    k_eval = float(np.mean([p[0] for p in per]))
    k_index = float(np.mean([p[1] for p in per])) if per and len(per[0]) > 1 else 0.0
    # deferred index pairs (engine.cpp launch): the index kernel runs first, so [0] holds the
    # value-class and index kernels and the pair sort, [1] the fills and the rest
    deferred = bool(per and len(per[0]) > 2 and per[0][2] == 1.0)
    if deferred:
        labels = ("mxp_vt_lookup/vt_eval + mxp_index_dtp_kernel + mxp_dtp_sort_kernel (deferred pairs, hit counters)",
                  "mxp_fill/vtfill/guard2/eval kernels + mxp_dtp_hits_kernel + the post-fill index launch (overflow list, next gate)")
    else:
        labels = ("phase1 (mxp_vt_classify/vt_eval/fill/vtfill/guard2/eval kernels)",
                  "mxp_index_kernel+mxp_inject_kernel + mxp_hits_kernel (streams the bitmap unless the kernels counted)")
    eval_ms = k_eval + k_index

    # algorithmic bytes of one evaluation: every referenced column read once per
    # request (kind u8 + value u64), the rule tables, the match bitmap and the error output written
    # (the error bitmap, or one flag byte per request in compact mode)
    n_cols = eng.ruleset_info()["columns"]
    prog_bytes = 16 * sum(eng.rule_vm_text(i).count("\n") for i in range(R)) + 4 * (R + 1)
    alg_bytes = N * n_cols * 9 + prog_bytes + N * Wd * 4 + (N if compact else N * Wd * 4)
    achieved = alg_bytes / (eval_ms * 1e-3) / 1e9
    traffic = measured_traffic(kind + ("q" if with_quota else ""), R, N)

    out = {
        "metric": metric,
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded %s workload; requests resident in HBM)" % kind.upper(),
        "config": {"workload": workload % (R, N),
                   "rules": R, "requests_per_gpu": N, "parallelism": "request-sharded dp%d" % world},
        "eval_ms": step_kernel_ms,
        "host_enqueue_ms_per_step": LAST_ENQUEUE_MS,
        "kernels_ms": {labels[0]: k_eval, labels[1]: k_index},
        "deferred_pairs": deferred,
        "pack_upload_s": t_pack,
        "error_output": "per-request flags (compact)" if compact else "error bitmap",
        "lds_bank_conflicts": lds_conflicts(kind),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("one evaluation: value classes (mxp_vt_lookup/vt_eval), guard index with deferred "
                                "pairs (mxp_index_dtp[_lite]_kernel), mxp_dtp_sort_kernel, bitmap fill merging the pairs "
                                "(mxp_fill_dtp / mxp_vtfill_lds), mxp_dtp_hits_kernel, post-fill mxp_index_kernel"
                                if deferred else
                                "one evaluation: value classes (mxp_vt_lookup/vt_eval), mxp_fill / vtfill / guard2 / eval "
                                "kernels (the groups each serves) + mxp_index_kernel (+ mxp_inject_kernel with dense "
                                "rules); traffic also counts mxp_hits_kernel when the hit counters are not fused"),
                     "alg_bytes_per_launch": alg_bytes, "alg_bytes_per_pair": alg_bytes / (N * R)},
    }
    if quota is not None:
        out["quota"] = {"keys": QUOTA_KEYS, "requests_per_gpu": int(quota[2][0].numel()),
                        "collective": "one all_reduce(sum) of hits[R] ++ quota_delta[K] per step"}
    hits = ctr.totals()[0]
    out["hits_total"] = int(hits.sum().item())
    if args.fresh_steps > 0 and not with_quota:
        def eval_db(dbx):
            if compact:
                dbx.eval_compact(d_match.data_ptr(), d_req_err.data_ptr(), scratch_hits.data_ptr(), sh)
            else:
                dbx.eval_hits(d_match.data_ptr(), d_err.data_ptr(), scratch_hits.data_ptr(), sh)
        out["fresh_batch"] = fresh_batch_block(eng, fresh_batches(kind, args.rules, args.requests, rank, world),
                                               eval_db, args.fresh_steps, stream, R, world)
    if args.e2e_reps > 0:
        out["end_to_end"] = end_to_end(eng, batch, R, args.e2e_reps)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        if kind == "c4":
            sample = W.c4_workload(n_rules=args.rules, n_requests=1 << 14, seed=4)[2]
            out["cpu_baseline"] = cpu_baseline(manifest, rules, sample, args.cpu_sample_seconds, args.cpu_threads,
                                               chunk=64)
        else:
            sample = W.c2_workload(n_rules=args.rules, n_requests=min(N, 1 << 18), seed=2)[2]
            out["cpu_baseline"] = cpu_baseline(manifest, rules, sample, args.cpu_sample_seconds, args.cpu_threads)
    db.free()
    del d_match, d_err, d_req_err
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from istio_amd import dist as D
    rank, world, local = D.world()
    # MXP_REHEARSE_MULTI=1: rehearsal of the N > 1 path on a one-GPU box -- every rank on cuda:0,
    # gloo collectives (RCCL refuses two ranks on one device); the line says so ("rehearsal")
    rehearse = world > 1 and os.environ.get("MXP_REHEARSE_MULTI") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from istio_amd import build
    build.build()

    if args.workload.startswith("c3"):
        return list_bench(args, rank, world, local)
    if args.workload == "c5-quota":
        return quota_bench(args, rank, world, local)
    kind = "c4" if args.workload == "c4" else "c2"
    out = predicate_bench(args, kind, rank, world, local, with_quota=args.workload == "c5")
    keys = ("metric", "value", "unit", "ms_per_step", "eval_ms", "kernels_ms", "deferred_pairs", "pack_upload_s",
            "fresh_batch", "end_to_end", "config", "roofline", "lds_bank_conflicts", "quota", "cpu_baseline")
    if args.workload == "c2" and not args.no_c4:
        # the representative config BASELINE.json quotes at 10k rules (configs[3]), driver-timed too
        c4 = predicate_bench(args, "c4", rank, world, local)
        out["c4"] = {k: c4[k] for k in keys if k in c4}
    if args.workload == "c2" and not args.no_c5:
        # configs[4]'s step: the C2 predicates + the memquota batch of the shard, then ONE all-reduce
        # of hits[R] ++ quota_delta[K] (at N = 1, the same step without the collective)
        a5 = argparse.Namespace(**vars(args))
        a5.e2e_reps = 0
        a5.no_cpu_baseline = True
        c5 = predicate_bench(a5, "c2", rank, world, local, with_quota=True)
        out["c5"] = {k: c5[k] for k in keys if k in c5}
    if args.workload == "c2" and not args.no_c3:
        # configs[2]: the three list kinds (100k entries, 1M lookups per GPU), driver-timed too
        a3 = argparse.Namespace(**vars(args))
        ckeys = ("metric", "value", "unit", "ms_per_step", "kernel_ms", "list_compile_s", "config", "roofline",
                 "lds_bank_conflicts", "cpu_baseline")
        out["c3"] = {}
        for k in ("c3-ip", "c3-str", "c3-regex"):
            r = list_bench(a3, rank, world, local, kind=k, emit=False)
            out["c3"][k[3:]] = {x: r[x] for x in ckeys if x in r}
    if rehearse:
        out["rehearsal"] = "%d ranks on one GPU over gloo: exercises the multi-rank step, not a scaling number" % world
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
