#!/usr/bin/env python3
"""Benchmark: request x rule predicate evaluations per second (BASELINE.json `metric`).

Headline workload (per GPU): the C2 rule family of BASELINE.json configs[1] (`destination.service ==
... && request.path.startsWith(...) && source.ip != ip(...)`) scaled to the metric's 10k rules, over
1M synthetic requests (Zipf(1.1) services) resident in HBM -- the per-GPU shard of configs[4]
(8 x MI355X, 8M requests).  A step = one evaluation of every rule against every request of every
shard (the full predicate bitmaps) + the per-rule hit counters, summed over the GPUs by the step's
one all-reduce.

The product path runs the step: a device group (include/mxp_group.h, istio_amd.engine.Group) -- ONE
process, as a Go Mixer is, holding one engine per GPU, each evaluating its contiguous shard, and
libmxp's own RCCL all-reduce (ncclCommInitAll communicators, one ncclAllReduce of hits[R] ++
quota_delta[K] per step).  At N = 1 nothing is reduced (the counters are the totals).

The default run also measures C4 (configs[3]: 10k Pilot-style route rules x 1M requests per GPU) as
the "c4" block (--no-c4: skip), C5 (configs[4]: the C2 step + the memquota batch routed to key owners
inside the group) as "c5" (--no-c5), and C3 (configs[2]: CIDR, case-insensitive string and regex
lists, 100k entries x 1M lookups per GPU) as "c3" (--no-c3).  Each predicate block also carries a
"fresh_batch" figure (a new batch uploaded from host memory and evaluated every step, PCIe-inclusive)
and an "end_to_end" Resolve figure.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rules R] [--requests N_PER_GPU]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
    python bench.py --workload c4 | c5 | c3-ip | c3-str | c3-regex | c5-quota [--devices 0,0]

Under torch.distributed.run (WORLD_SIZE = N) rank 0 drives the group over devices 0 .. N-1 and the
other ranks wait at a gloo barrier without touching a GPU: the data path's collective is libmxp's
RCCL all-reduce, not torch's.  --devices overrides the device list (e.g. 0,0: two members on one GPU,
the host reduction -- a rehearsal of the sharded path on a one-GPU box, not a scaling number).

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's default: 4).  A group member drives up to six streams (its
# evaluation, memquota, the engine's own, two copy streams, the packer's); at 4 queues the copy and
# packer streams shared one, so a fresh batch's H2D copies queued behind the previous batch's packer
# kernels: 1.29 -> 0.98 ms per fresh C2 step at 8 (profiles/r6_s11_fresh_hwq*.log; INTEGRATION.md
# sets it for the Mixer process the same way).  Read when HIP initialises; raised to 8 when the
# environment asks for fewer (the GPU boxes export the default 4), a larger value is kept.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 host link, spec (MI355X_MICROARCH.md)
QUOTA_KEYS = 1024
T0 = time.perf_counter()


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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--devices", default=None, help="comma-separated HIP devices of the group (default 0..N-1)")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rules", type=int, default=10000)
    p.add_argument("--requests", type=int, default=1 << 20, help="requests (C3: lookups) per GPU")
    p.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    p.add_argument("--cpu-threads", type=int, default=host_threads())
    p.add_argument("--list-cpu-seconds", type=float, default=4.0, help="CPU-baseline sample per C3 list kind")
    p.add_argument("--no-c3", action="store_true", help="default run: skip the extra C3 list block")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-c4", action="store_true", help="default run: skip the extra C4 block")
    p.add_argument("--no-c5", action="store_true", help="default run: skip the extra C5 block")
    p.add_argument("--workload", default="c2", choices=["c2", "c4", "c5", "c3-ip", "c3-str", "c3-regex", "c5-quota"],
                   help="c2 (default, the BASELINE metric; + C4 / C5 / C3 blocks); c4 route rules; c5 = C2 predicates "
                        "+ memquota with one combined all-reduce; C3 lists; c5-quota memquota alone")
    p.add_argument("--list-entries", type=int, default=100_000)
    p.add_argument("--e2e-reps", type=int, default=3, help="end-to-end resolve calls timed (median); 0 skips the end-to-end block (profiling sessions)")
    p.add_argument("--fresh-steps", type=int, default=10,
                   help="steps of the fresh-batch block (upload + evaluation of a new batch per step); 0 skips it")
    p.add_argument("--error-output", default="compact", choices=["compact", "bitmap"],
                   help="compact: per-request error flags (a Resolve's view); bitmap: the full error bitmap")
    p.add_argument("--wire", default="narrow", choices=["narrow", "wide"],
                   help="host batch format of the fresh-batch and end-to-end blocks: narrow (mxp_bag_batch2, "
                        "u32 ids and offsets, mxp_batch_upload2) or wide (mxp_bag_batch)")
    p.add_argument("--gen-procs", type=int, default=min(16, host_threads()),
                   help="processes generating the synthetic shards (before any GPU work)")
    return p.parse_args(argv)


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

    @staticmethod
    def _handle(stream):
        """A HIP stream handle from a raw int (mxp_group_stream) or a torch stream."""
        if stream is None or isinstance(stream, int):
            return stream or None
        return stream.cuda_stream

    def wait(self, stream):
        """`stream` waits for this event's record (hipStreamWaitEvent: an ordering, no host wait)."""
        h = StepEvent._hip
        h.hipStreamWaitEvent.argtypes = [self._ct.c_void_p, self._ct.c_void_p, self._ct.c_uint]
        if h.hipStreamWaitEvent(self._ct.c_void_p(self._handle(stream)), self.ev, 0):
            raise RuntimeError("hipStreamWaitEvent failed")

    def record(self, stream=None):
        if StepEvent._hip.hipEventRecord(self.ev, self._ct.c_void_p(self._handle(stream))):
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end):
        ms = self._ct.c_float()
        if StepEvent._hip.hipEventElapsedTime(self._ct.byref(ms), self.ev, end.ev):
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def __del__(self):
        if StepEvent._hip is not None and self.ev:
            StepEvent._hip.hipEventDestroy(self.ev)


def timed_loop(step, steps, warmup, world, stream, sync=None, events=True):
    """W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize; returns the
    slowest rank's seconds and the per-step HIP-event durations (ms) the step records on its stream.
    sync: the wait for all of the step's work (a group's mxp_group_sync: every member's streams);
    default torch.cuda.synchronize.  events=False (no GPU: the CPU tests of the step) records none."""
    import torch
    import torch.distributed as dist
    from istio_amd import dist as D
    if sync is None:
        sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    # (BENCH_FENCED_EVENTS=1: torch's default events instead, for same-box A/B of the fence's cost)
    mk = (lambda: torch.cuda.Event(enable_timing=True)) if os.environ.get("BENCH_FENCED_EVENTS") else StepEvent
    evs = [(mk(), mk()) if events else (None, None) for _ in range(steps)]
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
    ev_ms = [a.elapsed_time(b) for a, b in evs] if events else []
    # (world 1: this process times the whole job -- under torch.distributed.run rank 0 drives the
    # group while the other ranks wait at their barrier, so no collective here)
    return (D.max_over_ranks(elapsed) if world > 1 else elapsed), ev_ms


# ---------------------------------------------------------------------------------- synthetic data
def _gen(spec):
    """One synthetic shard (run in the generator pool, before any GPU work): ('c2' | 'c4', rules,
    n_total, lo, hi) -> BagBatch of requests [lo, hi) of the seeded n_total-request batch; ('c3-*',
    entries, lookups, seed) -> (entries, symbols)."""
    from istio_amd import workloads as W
    kind = spec[0]
    if kind == "c2":
        _, R, n_total, lo, hi = spec
        return W.c2_workload(n_rules=R, n_requests=n_total, seed=2, shard=(lo, hi))[2]
    if kind == "c4":
        _, R, n_total, lo, hi = spec
        return W.c4_workload(n_rules=R, n_requests=n_total, seed=4, shard=(lo, hi))[2]
    _, n_entries, n_look, seed = spec
    if kind == "c3-ip":
        return W.c3_ip_list(n_entries=n_entries, n_lookups=n_look, seed=seed)
    if kind == "c3-str":
        return W.c3_string_list(n_entries=n_entries, n_lookups=n_look, seed=seed)
    return W.c3_regex_list(n_patterns=min(n_entries, 10_000), n_lookups=n_look, seed=seed)


class Data:
    """Every synthetic input of the run, generated up front in a process pool (before the GPU is
    touched: the pool forks this process).  Predicate shards: member k's requests of ONE seeded batch
    of G x --requests requests (configs[4]: 8 x 1M), contiguous (mxp_group_shard_bounds); the two
    fresh-batch sets are the next two such batches of the same seeded stream."""

    def __init__(self, args, G, kinds):
        from istio_amd import dist as D
        self.G, self.per = G, args.requests
        n_total = args.requests * G
        specs = []
        for kind in ("c2", "c4"):
            if kind not in kinds:
                continue
            fresh = args.fresh_steps > 0
            for rep in range(3 if fresh else 1):
                for k in range(G):
                    lo, hi = D.shard_bounds(n_total, k, G)
                    nt = 3 * n_total if fresh else n_total
                    specs.append(((kind, rep, k), (kind, args.rules, nt, lo + rep * n_total, hi + rep * n_total)))
        for kind in ("c3-ip", "c3-str", "c3-regex"):
            if kind in kinds:
                for k in range(G):
                    specs.append(((kind, 0, k), (kind, args.list_entries, args.requests, 3 + 1000 * k)))
        self.items = {}
        procs = max(1, min(args.gen_procs, len(specs)))
        if procs > 1:
            import multiprocessing as mp
            with mp.get_context("fork").Pool(procs) as pool:
                for key, val in zip([s[0] for s in specs], pool.map(_gen, [s[1] for s in specs], chunksize=1)):
                    self.items[key] = val
        else:
            for key, spec in specs:
                self.items[key] = _gen(spec)

    def shards(self, kind, rep=0):
        return [self.items[(kind, rep, k)] for k in range(self.G)]


def rule_set(kind, n_rules):
    from istio_amd import workloads as W
    if kind == "c4":
        manifest, rules, _ = W.c4_workload(n_rules=n_rules, n_requests=1, seed=4)
        return manifest, rules
    manifest, _, _ = W.c2_workload(n_rules=n_rules, n_requests=1, seed=2)
    return manifest, W.c2_rules(n_rules, seed=2)[0]


def batch_h2d_bytes(batch):
    """Bytes of the host columnar batch mxp_batch_upload copies to the device (Go-owned bags)."""
    n = sum(k.nbytes for k in batch.kinds) + sum(v.nbytes for v in batch.values)
    return int(n + batch.str_blob.nbytes + batch.str_offsets.nbytes + batch.time_sec.nbytes + batch.time_nsec.nbytes
               + batch.map_offsets.nbytes + batch.map_keys.nbytes + batch.map_values.nbytes)


# ---------------------------------------------------------------------------------- blocks
def make_group(devices):
    from istio_amd.engine import Group
    return Group(devices)


def group_step(g, gb, quota=None, s0=None):
    """The bench step on a device group: every member evaluates its shard with the hit
    counters fused into the step's hits[R]; with `quota` = (GroupQuota, batch, [now]) each key owner's
    memquota replay runs beside it (its per-key deltas into quota_delta[K]); then the step's ONE
    all-reduce of hits[R] ++ quota_delta[K] (mxp_group_reduce: RCCL, nothing at one member).  ev0 / ev1
    bracket member 0's work on its stream s0."""
    def step(ev0=None, ev1=None):
        if ev0 is not None:
            ev0.record(s0)
        g.eval(gb)
        if quota is not None:
            q, qb, now = quota
            q.eval(qb, now[0])
            now[0] += 10**8
        g.reduce()
        if ev1 is not None:
            ev1.record(s0)
    return step


def host_sets(shard_sets, wire):
    """Pinned host copies of shard sets (a binding's reused packing arenas), wide
    (BagBatch) or narrow (bags.NarrowBatch); (sets, bytes over the link per set, keep-alive)."""
    from istio_amd.engine import pinned_batch, pinned_narrow
    mk = pinned_narrow if wire == "narrow" else pinned_batch
    made = [[mk(b) for b in shards] for shards in shard_sets]
    sets = [[b for b, _ in m] for m in made]
    size = (lambda b: b.wire_bytes()) if wire == "narrow" else batch_h2d_bytes
    return sets, [sum(size(b) for b in st) for st in sets], made


def upload_set(g, st, wire, no_wait):
    return g.upload2(st, no_wait=no_wait) if wire == "narrow" else g.upload(st, no_wait=no_wait)


def fresh_batch_block(g, fresh_sets, steps, n_rules, wire="narrow"):
    """Every step takes a NEW set of shards from host memory, double-buffered: mxp_group_upload of set
    k + 1 with MXP_UPLOAD_NO_WAIT (its H2D copies queued on every member and the shards checked; the
    device packers run after them), then the evaluation of set k (its first evaluation finishes its
    packing: class tables, string heads, dictionary; enqueued); a host set is refilled only after the
    previous upload of it has been copied (mxp_group_batch_wait_copied), two steps back.  The two host
    sets alternate; a device set is freed three steps after its evaluation.  PCIe-inclusive.  The host
    shards live in pinned memory (mxp_host_alloc), as a binding's reused packing arenas do
    (INTEGRATION.md 2e): their copies are DMA at the link's rate."""
    import numpy as np
    sets, h2d, _keep = host_sets(fresh_sets, wire)
    keep, up_s, pending, copying = [], [], [], []

    def one(k):
        if len(copying) >= len(sets):  # (this step's host set was uploaded len(sets) steps ago)
            copying.pop(0).wait_copied()
        t0 = time.perf_counter()
        gb = upload_set(g, sets[k % len(sets)], wire, True)  # (copies queued, shards checked)
        up_s.append(time.perf_counter() - t0)
        copying.append(gb)
        if pending:  # (the previous set, uploaded one step ago)
            prev = pending.pop()
            g.eval(prev)
            keep.append(prev)
            if len(keep) > 3:
                keep.pop(0).free()
        pending.append(gb)
    for k in range(3):  # warm-up (allocations)
        one(k)
    g.sync()
    up_s.clear()
    t0 = time.perf_counter()
    for k in range(steps):  # (k uploads and k evaluations)
        one(k)
    g.sync()
    dt = (time.perf_counter() - t0) / steps
    while pending:
        g.eval(pending[0])
        keep.append(pending.pop())
    g.sync()
    copying.clear()
    while keep:
        keep.pop(0).free()
    N = sum(b.n for b in sets[0])
    up = float(np.mean(up_s))
    bytes_step = float(np.mean([h2d[k % len(sets)] for k in range(steps)]))
    G = len(sets[0])
    return {"ms_per_step": dt * 1e3, "upload_ms": up * 1e3, "requests_per_s": N / dt,
            "pairs_per_s": N * n_rules / dt, "steps": steps, "h2d_bytes_per_batch": int(bytes_step / G),
            "roofline": {"bound": "pcie", "achieved": bytes_step / G / dt / 1e9, "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                         "frac": bytes_step / G / dt / 1e9 / PCIE_PEAK_GBS, "traffic": None,
                         "kernel": "mxp_batch_upload: H2D copy of the host columnar batch + the device packer "
                                   "(intern, gather, pool, pre-tables, value-class dictionary, heads); "
                                   "achieved = batch bytes per GPU / step wall time (upload + evaluation, pipelined)"},
            "upload_call_gbs": bytes_step / up / 1e9,
            "host_memory": "pinned (mxp_host_alloc arenas)", "wire": wire,
            "path": "host columnar shards (a new batch every step; %s) -> mxp_group_upload%s (set k + 1) -> "
                    "mxp_group_eval (set k: compact errors, fused hit counters); wall time per step, PCIe-inclusive" % (
                        "mxp_bag_batch2: u32 ids and offsets" if wire == "narrow" else "mxp_bag_batch",
                        "2" if wire == "narrow" else "")}


def end_to_end(g, shard_sets, n_rules, reps, wire="narrow"):
    """The whole Check-path call from Go-owned bags to action lists: the host
    columnar shards -> mxp_group_resolve_batch (per member: device packing and interning, evaluation of
    every pair, per-request resolution and action-list gather on the device) -> status / first-error
    rule / selected rules of the whole batch back in host memory.  Every rule sits in the default
    namespace with one variety, so each request's action list is every rule whose predicate holds
    (resolver.go:202-238).  PCIe-inclusive; not `value` (whose inputs are resident in HBM).

    ms_per_batch: one call (median of reps).  pipelined: what a micro-batcher with two packing arenas
    sustains -- batch k + 1 uploaded (mxp_group_upload, MXP_UPLOAD_NO_WAIT) before batch k's Resolve
    (mxp_group_resolve_uploaded), so k + 1's copies and device packing overlap k's evaluation, resolve
    kernels and downloads; the three shard sets alternate."""
    import numpy as np
    from istio_amd.engine import PinnedArena
    g.set_resolver("destination.service", "istio-system", ["istio-system"] * n_rules,
                   np.ones(n_rules, dtype=np.uint32), np.zeros(n_rules, dtype=np.uint8),
                   np.zeros(n_rules, dtype=np.uint8))
    sets, h2d, _keep = host_sets(shard_sets, wire)  # (the binding's packing arenas)
    shards = sets[0]
    n = sum(b.n for b in shards)
    ids16 = n_rules <= 65536  # MXP_RESOLVE_IDS_U16
    narrow = wire == "narrow"

    def resolve(st, cap=0, out=None):  # one call from host bags: upload (narrow) + Resolve, or the one-shot call
        if narrow:
            # (the upload returns once its copies are queued -- MXP_UPLOAD_NO_WAIT, as a binding calls
            # it -- and the Resolve's first evaluation orders itself after them; BENCH_E2E_WAIT=1: the
            # upload waits for its copies first, A/B)
            return g.resolve_arrays(None, 0, cap or max(16, 4 * n), ids16=ids16, out=out,
                                    uploaded=upload_set(g, st, wire, not os.environ.get("BENCH_E2E_WAIT")))
        return g.resolve_arrays(st, 0, cap, ids16=ids16, out=out)
    # list sizes (the one-shot call from the wide form: an uploaded batch's Resolve cannot retry when
    # its ids do not fit), then a warm-up of the measured call (allocations)
    caps = [int(g.resolve_arrays([getattr(b, "batch", b) for b in st], 0, ids16=ids16)[2][-1]) for st in sets]
    cap = max(16, 2 * max(caps))
    for st in sets:
        resolve(st, cap)
    arena = PinnedArena(n * 13 + 8 + cap * 2 + 4 * 64)
    out = (arena.empty(n, np.uint8), arena.empty(n, np.uint32), arena.empty(n + 1, np.uint64),
           arena.empty(cap, np.uint16 if ids16 else np.uint32))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        status, _, off, _ = resolve(shards, cap, out)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    sel_bytes = int(off[-1]) * (2 if ids16 else 4)
    err_requests = int((status == 3).sum())
    selected = float(off[-1]) / max(n, 1)
    # pipelined: batch k's evaluation submitted (mxp_group_resolve_submit), batch k + 1 uploaded while
    # it runs -- the upload's host checks and packing overlap the device -- then k finished
    # (BENCH_PIPE_SUBMIT=0: the one-call Resolve after the upload, the round-5 order, A/B)
    split = os.environ.get("BENCH_PIPE_SUBMIT", "1") != "0"
    steps = max(3 * reps, 6)
    nxt = upload_set(g, sets[0], wire, True)
    t0 = time.perf_counter()
    for k in range(steps):
        cur = nxt
        job = g.resolve_submit(cur, 0, ids16=ids16) if split else None
        if k + 1 < steps:
            nxt = upload_set(g, sets[(k + 1) % len(sets)], wire, True)
        if split:
            g.resolve_finish(job, cap, out=out)
        else:
            g.resolve_arrays(None if narrow else sets[k % len(sets)], 0, cap, ids16=ids16, out=out, uploaded=cur)
    t_pipe = (time.perf_counter() - t0) / steps
    G = len(shards)
    return {"pairs_per_s": n * n_rules / t, "requests_per_s": n / t, "ms_per_batch": t * 1e3,
            "requests_per_gpu": n // G, "reps": reps, "selected_per_request": selected,
            "pred_error_requests": err_requests, "rule_ids": "u16" if ids16 else "u32",
            "action_list_bytes": sel_bytes, "action_list_ms_at_50GBps": sel_bytes / G / 50e9 * 1e3,
            "x_action_list_at_50GBps": t * 1e3 / max(sel_bytes / G / 50e9 * 1e3, 1e-9),
            "pipelined": {"ms_per_batch": t_pipe * 1e3, "requests_per_s": n / t_pipe, "pairs_per_s": n * n_rules / t_pipe,
                          "batches": steps, "x_action_list_at_50GBps": t_pipe * 1e3 / max(sel_bytes / G / 50e9 * 1e3, 1e-9),
                          "path": ("mxp_group_resolve_submit(batch k), mxp_group_upload(batch k + 1, MXP_UPLOAD_NO_WAIT), "
                                   "mxp_group_resolve_finish(batch k)" if split else
                                   "mxp_group_upload(batch k + 1, MXP_UPLOAD_NO_WAIT) then mxp_group_resolve_uploaded(batch k)")
                                  + "; three pinned shard sets alternating; wall time per batch"},
            "host_memory": "pinned shards and outputs (mxp_host_alloc arenas)", "wire": wire,
            "h2d_bytes_per_batch": int(h2d[0] / G),
            "path": ("host columnar shards -> %s -> host action lists of the whole batch (per member: device pack + "
                     "namespaces + compact evaluation + first errors from the records + device scan + action-list "
                     "gather); median of reps, PCIe-inclusive" % (
                         "mxp_group_upload2 (narrow: u32 ids and offsets) + mxp_group_resolve_uploaded" if narrow
                         else "mxp_group_resolve_batch"))}


def predicate_bench(args, kind, devices, data, with_quota=False):
    """One predicate workload (c2 / c4) over the group's shards (--requests per GPU); returns the
    result dict.  Step: group_step (every member's evaluation with fused hit counters, optionally the
    memquota batch routed to key owners, then the step's one all-reduce)."""
    import numpy as np
    from istio_amd import workloads as W
    from istio_amd.engine import key_owners

    G = len(devices)
    manifest, rules = rule_set(kind, args.rules)
    shards = data.shards(kind)
    if kind == "c4":
        metric, workload = ("request x rule predicate evals/sec at 10k rules (C4 route rules)",
                            "C4 Pilot-style route rules R=%d, %d requests per GPU (configs[3])")
    else:
        metric, workload = ("request x rule predicate evals/sec at 10k rules",
                            "C2 rules scaled to R=%d, %d requests per GPU (configs[1] family, configs[4] shard)")
        if with_quota:
            workload = "C5: C2 rules R=%d, %d requests per GPU + memquota (configs[4])"
    g = make_group(devices)
    g.set_vocabulary(manifest)
    st = g.compile(rules)
    assert (st == 0).all()
    t_pack = time.perf_counter()
    gb = g.upload(shards)
    t_pack = time.perf_counter() - t_pack
    R, N = len(rules), shards[0].n
    N_all = sum(b.n for b in shards)
    compact = args.error_output == "compact"
    quota = None
    if with_quota:
        # ONE global arrival stream of quota requests (G x --requests), routed to the keys' owners
        # inside the group (mxp_group_quota_upload; owners by expected load, mxp_group_key_owners)
        mx, vd, keys, amounts, be = W.quota_workload(n_keys=QUOTA_KEYS, n_requests=args.requests * G, seed=5)
        q = g.quota_create(mx, vd, key_owners(W.quota_key_weights(QUOTA_KEYS), G))
        qb = q.upload(keys, amounts, be)
        quota = (q, qb, [1_500_000_000 * 10**9])
    s0 = g.stream(0)
    if compact:
        step = group_step(g, gb, quota, s0)
    else:
        def step(ev0=None, ev1=None):
            if ev0 is not None:
                ev0.record(s0)
            g.eval(gb, err_bitmap=True)
            if quota is not None:
                quota[0].eval(quota[1], quota[2][0])
                quota[2][0] += 10**8
            g.reduce()
            if ev1 is not None:
                ev1.record(s0)
    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, 1, None, sync=g.sync)
    step_kernel_ms = float(np.mean(ev_ms))
    value = N_all * R * args.steps / elapsed
    hits, delta = g.counters(QUOTA_KEYS if quota else 0)
    hits_total = int(hits.sum())

    # per-kernel durations of member 0 (HIP events recorded by libmxp around each launch on its stream),
    # in a separate pass so the timed region above carries no extra synchronisation
    e0 = g.engine(0)
    e0.set_timing(True)
    per = []
    for _ in range(args.steps):
        g.eval(gb, err_bitmap=not compact)
        per.append(e0.kernel_times(3))
    e0.set_timing(False)
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

    # algorithmic bytes of one evaluation on one GPU: every referenced column read
    # once per request (kind u8 + value u64), the rule tables, the match bitmap and the error output
    # written (the error bitmap, or one flag byte per request in compact mode)
    Wd = (R + 31) // 32
    n_cols = e0.ruleset_info()["columns"]
    prog_bytes = 16 * sum(e0.rule_vm_text(i).count("\n") for i in range(R)) + 4 * (R + 1)
    alg_bytes = N * n_cols * 9 + prog_bytes + N * Wd * 4 + (N if compact else N * Wd * 4)
    achieved = alg_bytes / (eval_ms * 1e-3) / 1e9
    traffic = measured_traffic(kind + ("q" if with_quota else ""), R, N)

    out = {
        "metric": metric,
        "value": value,
        "unit": "pairs/s",
        "n_gpus": G,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded %s workload; requests resident in HBM)" % kind.upper(),
        "config": {"workload": workload % (R, N),
                   "rules": R, "requests_per_gpu": N, "parallelism": "request-sharded dp%d" % G},
        "group": {"devices": list(devices), "reduce": ["none", "rccl", "host"][g.reduce_mode],
                  "note": g.note or None, "process": "one process drives every GPU (mxp_group)"},
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
        "hits_total": hits_total,
    }
    if quota is not None:
        out["quota"] = {"keys": QUOTA_KEYS, "requests": int(quota[1].n),
                        "requests_per_gpu": [quota[1].requests(k) for k in range(G)],
                        "quota_delta_abs_total": int(np.abs(delta).sum()),
                        "collective": "one all-reduce of hits[R] ++ quota_delta[K] per step (mxp_group_reduce)"}
    if args.fresh_steps > 0 and not with_quota:
        progress("%s fresh batches" % kind)
        out["fresh_batch"] = fresh_batch_block(g, [data.shards(kind, 1), data.shards(kind, 2)], args.fresh_steps, R,
                                               args.wire)
    if args.e2e_reps > 0 and not with_quota:
        sets = [shards] + ([data.shards(kind, 1), data.shards(kind, 2)] if args.fresh_steps > 0 else [])
        progress("%s end to end" % kind)
        out["end_to_end"] = end_to_end(g, sets, R, args.e2e_reps, args.wire)
    gb.free()
    if quota is not None:
        quota[1].free()
    quota = None
    g.close()
    if not args.no_cpu_baseline and G == 1:
        if kind == "c4":
            sample = W.c4_workload(n_rules=args.rules, n_requests=1 << 14, seed=4)[2]
            out["cpu_baseline"] = cpu_baseline(manifest, rules, sample, args.cpu_sample_seconds, args.cpu_threads,
                                               chunk=64)
        else:
            sample = W.c2_workload(n_rules=args.rules, n_requests=min(N, 1 << 18), seed=2)[2]
            out["cpu_baseline"] = cpu_baseline(manifest, rules, sample, args.cpu_sample_seconds, args.cpu_threads)
    return out


def list_bench(args, devices, data, kind=None, emit=True):
    """C3 (BASELINE configs[2]): 100k-entry CIDR / string / regex lists replicated on every member,
    --requests lookups per GPU resident in HBM; one step = HandleListEntry for every lookup
    (mxp_group_list_check_device: one kernel per member).  Returns the result dict."""
    import numpy as np
    import torch
    from istio_amd.engine import ListHandle
    kind = kind or args.workload
    G = len(devices)
    per = data.shards(kind)
    entries = per[0][0]
    etype = {"c3-ip": ListHandle.IP_ADDRESSES, "c3-str": ListHandle.CASE_INSENSITIVE_STRINGS}.get(kind, ListHandle.REGEX)
    g = make_group(devices)
    t0 = time.perf_counter()
    gl = g.list_create(etype, entries)
    t_compile = time.perf_counter() - t0
    d_syms, d_offs, d_codes, ns, algs = [], [], [], [], []
    for k, (_, syms) in enumerate(per):
        bs = [x.encode() for x in syms]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        blob = np.frombuffer(b"".join(bs) + bytes(16), dtype=np.uint8)
        dev = torch.device("cuda", devices[k])
        d_syms.append(torch.from_numpy(blob.copy()).to(dev))
        d_offs.append(torch.from_numpy(off.view(np.int64).copy()).to(dev))
        d_codes.append(torch.empty(len(bs), dtype=torch.int32, device=dev))
        ns.append(len(bs))
        algs.append(int(off[-1]) + 8 * (len(bs) + 1) + 4 * len(bs))  # symbol bytes + offsets read, one code written each
    torch.cuda.synchronize()
    s0 = g.stream(0)
    ptrs = ([t.data_ptr() for t in d_syms], [t.data_ptr() for t in d_offs], [t.data_ptr() for t in d_codes])

    def step(e0=None, e1=None):
        if e0 is not None:
            e0.record(s0)
        gl.check_device(ptrs[0], ptrs[1], ns, ptrs[2])
        if e1 is not None:
            e1.record(s0)
    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, 1, None, sync=g.sync)
    kernel_ms = float(np.mean(ev_ms))
    n, alg = ns[0], algs[0]
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    # the kernel the step launches (lists.cpp mxp_list_check_device): CIDR lookups regrouped by
    # address family, string lookups by the register window, regex lists with their automata staged
    # in LDS unless MXP_LIST_LDS=0
    kname = {"c3-ip": "mxp_list_ip_kernel", "c3-str": "mxp_list_str_kernel"}.get(
        kind, "mxp_list_rx_kernel" if os.environ.get("MXP_LIST_LDS", "1") != "0" else "mxp_list_kernel")
    out = {"metric": "list-adapter lookups/sec (%s, %d entries)" % (kind, gl.member(0).num_entries()),
           "value": sum(ns) * args.steps / elapsed, "unit": "lookups/s", "n_gpus": G, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (seeded C3 %s list and lookups; symbols resident in HBM)" % kind[3:],
           "config": {"workload": "C3 %s list, %d entries, %d lookups per GPU (configs[2])" % (kind[3:], len(entries), n),
                      "entries": len(entries), "lookups_per_gpu": n, "parallelism": "lookup-sharded dp%d" % G},
           "kernel_ms": kernel_ms, "list_compile_s": t_compile,
           "lds_bank_conflicts": lds_conflicts(kind),
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": measured_traffic(kind, args.list_entries, n),
                        "kernel": kname, "alg_bytes_per_launch": alg}}
    del d_syms, d_offs, d_codes, gl
    g.close()
    if not args.no_cpu_baseline and G == 1:
        out["cpu_baseline"] = list_cpu_baseline(kind, entries, per[0][1], args.list_cpu_seconds, args.cpu_threads)
    if emit:
        print(json.dumps(out))
    return out


def quota_bench(args, devices):
    """C5 memquota (BASELINE configs[4]): K = 1024 quota keys replicated on every member, each owned by
    one (mxp_group_key_owners), one global arrival stream of --requests x G quota requests routed to
    the owners inside the group (mxp_group_quota_upload); a step = every owner's batched HandleQuota
    (sort by key + per-key replay) and the all-reduce of the per-key deltas."""
    import numpy as np
    from istio_amd import workloads as W
    from istio_amd.engine import key_owners
    G = len(devices)
    mx, vd, keys, amounts, be = W.quota_workload(n_keys=QUOTA_KEYS, n_requests=args.requests * G, seed=5)
    g = make_group(devices)
    q = g.quota_create(mx, vd, key_owners(W.quota_key_weights(QUOTA_KEYS), G))
    qb = q.upload(keys, amounts, be)
    s0 = g.stream(0)
    now = [1_500_000_000 * 10**9]

    def step(e0=None, e1=None):
        if e0 is not None:
            e0.record(s0)
        q.eval(qb, now[0])
        g.reduce()
        if e1 is not None:
            e1.record(s0)
        now[0] += 10**8
    elapsed, ev_ms = timed_loop(step, args.steps, args.warmup, 1, None, sync=g.sync)
    kernel_ms = float(np.mean(ev_ms))
    n0 = qb.requests(0)
    alg = n0 * (4 + 8 + 1 + 8)  # key, amount, best effort read; granted written
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    out = {"metric": "memquota HandleQuota requests/sec (%d keys)" % QUOTA_KEYS,
           "value": len(keys) * args.steps / elapsed,
           "unit": "requests/s", "n_gpus": G, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "int64", "data": "synthetic (seeded C5 quota requests routed to key owners in the group; resident in HBM)",
           "config": {"workload": "C5 memquota, %d keys, %d requests per GPU (configs[4])" % (QUOTA_KEYS, args.requests),
                      "keys": QUOTA_KEYS, "requests_per_gpu": [qb.requests(k) for k in range(G)],
                      "parallelism": "key-owner-sharded dp%d" % G},
           "kernel_ms": kernel_ms,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                        "kernel": "counting sort by key (mxp_quota_hist / binscan / scatter) + mxp_quota_kernel",
                        "alg_bytes_per_launch": alg}}
    qb.free()
    del q
    g.close()
    if not args.no_cpu_baseline and G == 1:
        # the C restatement (oracle/memquota_oracle.c): the same batches, keys in parallel on the
        # host's cores (each key's requests sequential, as the reference's mutex runs them)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import memquota as M
        ref = M.CMemquota(mx, vd)
        t0 = time.perf_counter()
        done, t_ns, n = 0, 1_500_000_000 * 10**9, len(keys)
        while done == 0 or (time.perf_counter() - t0 < args.cpu_sample_seconds and done < 64 * n):
            ref.handle_batch(keys, amounts, be, t_ns, threads=args.cpu_threads)
            done += n
            t_ns += 10**8
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": done / dt, "unit": "requests/s", "cores": args.cpu_threads,
                               "host_cpus": os.cpu_count(), "kind": "port",
                               "sample": "%d requests (%d batches of %d, %.1fs), memquota C restatement, keys in "
                                         "parallel on %d threads" % (done, done // n, n, dt, args.cpu_threads)}
    return out


def list_cpu_baseline(kind, entries, syms, seconds, threads):
    """The list restatements timed on host cores, compiled and multi-threaded (OpenMP over the
    lookups): the IP list is the reference's linear IPNet scan (ipList.go:77-92); case-insensitive
    strings a hash set after Go's strings.ToUpper (stringList.go:51-80, a Go map); regexes the Go
    regexp restatement, patterns tried in order until one matches (regexList.go:26-33)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lists as L
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


def progress(what):
    """A progress note on stderr (the JSON line is stdout's only line): a long multi-GPU run keeps
    writing while its blocks run."""
    print("bench: %s (%.0f s)" % (what, time.perf_counter() - T0), file=sys.stderr, flush=True)


def run(args, devices):
    """Every block of the run over the group `devices`; returns the line (a dict)."""
    progress("generating inputs for %d device(s)" % len(devices))
    kinds = set()
    wl = args.workload
    if wl in ("c2", "c5"):
        kinds.add("c2")
    if wl == "c4" or (wl == "c2" and not args.no_c4):
        kinds.add("c4")
    if wl.startswith("c3"):
        kinds.add(wl)
    if wl == "c2" and not args.no_c3:
        kinds |= {"c3-ip", "c3-str", "c3-regex"}
    data = Data(args, len(devices), kinds) if wl != "c5-quota" else None
    if wl.startswith("c3"):
        return list_bench(args, devices, data, emit=False)
    if wl == "c5-quota":
        return quota_bench(args, devices)
    kind = "c4" if wl == "c4" else "c2"
    progress("%s block" % wl)
    out = predicate_bench(args, kind, devices, data, with_quota=wl == "c5")
    keys = ("metric", "value", "unit", "ms_per_step", "eval_ms", "kernels_ms", "deferred_pairs", "pack_upload_s",
            "fresh_batch", "end_to_end", "config", "group", "roofline", "lds_bank_conflicts", "quota", "cpu_baseline",
            "hits_total")
    if wl == "c2" and not args.no_c4:
        # the representative config BASELINE.json quotes at 10k rules (configs[3]), driver-timed too
        progress("c4 block")
        c4 = predicate_bench(args, "c4", devices, data)
        out["c4"] = {k: c4[k] for k in keys if k in c4}
    if wl == "c2" and not args.no_c5:
        # configs[4]'s step: the C2 predicates + the memquota batch routed to its key owners, then ONE
        # all-reduce of hits[R] ++ quota_delta[K] (at N = 1, the same step without the collective)
        a5 = argparse.Namespace(**vars(args))
        a5.e2e_reps = 0
        a5.no_cpu_baseline = True
        progress("c5 block")
        c5 = predicate_bench(a5, "c2", devices, data, with_quota=True)
        out["c5"] = {k: c5[k] for k in keys if k in c5}
    if wl == "c2" and not args.no_c3:
        # configs[2]: the three list kinds (100k entries, --requests lookups per GPU), driver-timed too
        ckeys = ("metric", "value", "unit", "ms_per_step", "kernel_ms", "list_compile_s", "config", "roofline",
                 "lds_bank_conflicts", "cpu_baseline")
        out["c3"] = {}
        for k in ("c3-ip", "c3-str", "c3-regex"):
            progress("%s block" % k)
            r = list_bench(args, devices, data, kind=k, emit=False)
            out["c3"][k[3:]] = {x: r[x] for x in ckeys if x in r}
    return out


def main():
    args = parse()
    if os.environ.get("MXP_BENCH_WATCHDOG"):  # (debugging: every thread's Python stack every N s)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["MXP_BENCH_WATCHDOG"]), repeat=True, file=sys.stderr)
    from istio_amd import dist as D
    rank, world, _ = D.world()
    n_gpus = world if world > 1 else args.gpus
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(n_gpus))
    if world > 1:
        # launched by torch.distributed.run: rank 0 drives the whole group from one process (as a Go
        # Mixer does); the other ranks touch no GPU and wait for it here (gloo: control only)
        import torch.distributed as dist
        dist.init_process_group("gloo")
        if rank != 0:
            dist.barrier()
            dist.destroy_process_group()
            return
    from istio_amd import build
    build.build()
    out = run(args, devices)
    if out is not None:
        if len(set(devices)) < len(devices):
            out["rehearsal"] = ("%d members on %d GPU(s), host reduction: exercises the sharded step, not a scaling "
                                "number" % (len(devices), len(set(devices))))
        if world > 1:
            out["launch"] = "torch.distributed.run x %d: rank 0 drives the %d-GPU group, ranks 1..%d idle" % (
                world, len(devices), world - 1)
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
