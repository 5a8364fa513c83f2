"""Synthetic, seeded workloads for the Mixer Check predicate path (BASELINE.json configs).

  C1 (seed 1)  Bookinfo / testdata Mixer rules + `true` rules over 10k bags.
  C2 (seed 2)  `destination.service == ... && request.path.startsWith(...) && source.ip != ip(...)`
               rules (1k in the config; the bench scales the same generator to 10k rules), 64k requests
               with Zipf(1.1) services.
  fuzz         random well- and ill-typed expressions over the reference's default test vocabulary
               (mixer/pkg/il/testing/tests.go:2414-2489) and random bags with missing and wrongly-typed
               values -- the parity stress test.

All generation is numpy-seeded and deterministic.  The vocabulary of C1/C2 is the attribute manifest
of mixer/testdata/config/attributes.yaml (names and value types only).
"""
from __future__ import annotations

import numpy as np

from .bags import (ABSENT, BOOL, BYTES, DOUBLE, DURATION, INT64, STRING, STRING_MAP, TIMESTAMP, BagBatch,
                   GoDuration, GoFloat64, GoInt64, GoOther, GoTime)

# mixer/testdata/config/attributes.yaml
TESTDATA_MANIFEST = {
    "origin.ip": "IP_ADDRESS", "origin.uid": "STRING", "origin.user": "STRING", "request.headers": "STRING_MAP",
    "request.id": "STRING", "request.host": "STRING", "request.method": "STRING", "request.path": "STRING",
    "request.reason": "STRING", "request.referer": "STRING", "request.scheme": "STRING", "request.size": "INT64",
    "request.time": "TIMESTAMP", "request.useragent": "STRING", "response.code": "INT64",
    "response.duration": "DURATION", "response.headers": "STRING_MAP", "response.size": "INT64",
    "response.time": "TIMESTAMP", "source.uid": "STRING", "source.user": "STRING", "target.uid": "STRING",
    "destination.uid": "STRING", "connection.id": "STRING", "connection.received.bytes": "INT64",
    "connection.received.bytes_total": "INT64", "connection.sent.bytes": "INT64",
    "connection.sent.bytes_total": "INT64", "connection.duration": "DURATION", "context.protocol": "STRING",
    "context.timestamp": "TIMESTAMP", "context.time": "TIMESTAMP", "api.service": "STRING",
    "api.version": "STRING", "api.operation": "STRING", "api.protocol": "STRING",
    "request.auth.principal": "STRING", "request.auth.audiences": "STRING", "request.auth.presenter": "STRING",
    "request.api_key": "STRING", "source.ip": "IP_ADDRESS", "source.labels": "STRING_MAP",
    "source.name": "STRING", "source.namespace": "STRING", "source.service": "STRING",
    "source.serviceAccount": "STRING", "target.ip": "IP_ADDRESS", "target.labels": "STRING_MAP",
    "target.name": "STRING", "target.namespace": "STRING", "target.service": "STRING",
    "target.serviceAccount": "STRING", "destination.ip": "IP_ADDRESS", "destination.labels": "STRING_MAP",
    "destination.name": "STRING", "destination.namespace": "STRING", "destination.service": "STRING",
    "destination.serviceAccount": "STRING",
}

# mixer/pkg/il/testing/tests.go:2414-2489 (defaultAttrs)
DEFAULT_TEST_MANIFEST = {
    "ai": "INT64", "ab": "BOOL", "as": "STRING", "ad": "DOUBLE", "ar": "STRING_MAP", "adur": "DURATION",
    "at": "TIMESTAMP", "aip": "IP_ADDRESS", "bi": "INT64", "bb": "BOOL", "bs": "STRING", "bd": "DOUBLE",
    "br": "STRING_MAP", "bdur": "DURATION", "bt": "TIMESTAMP", "t1": "TIMESTAMP", "t2": "TIMESTAMP",
    "bip": "IP_ADDRESS", "b1": "BOOL", "b2": "BOOL", "sm": "STRING_MAP",
}

# Bookinfo / testdata rule selectors
BOOKINFO_RULES = [
    'destination.labels["app"] == "ratings" && source.labels["app"]=="reviews" && source.labels["version"] == "v3"',
    'destination.labels["app"] == "details" && source.user == "cluster.local/ns/default/sa/bookinfo-productpage"',
    'request.headers["x-user"] == ""',
    '(destination.labels["app"]|"unknown") == "ratings"',
    'request.headers["clnt"] == "abc"',
    'destination.service == "foo.default.svc.cluster.local" && source.ip != ip("10.11.12.13")',
    'destination.service == "bar.default.svc.cluster.local" && source.user != "tcp-test-user"',
    'context.protocol == "tcp"',
]


def _ip4(a, b, c, d):
    return bytes([a, b, c, d])


def c1_workload(n_bags=10000, seed=1, n_true_rules=8):
    """Bookinfo rules (+ `true` rules) and n_bags bags with ~5% missing attributes."""
    rng = np.random.default_rng(seed)
    rules = list(BOOKINFO_RULES) + ["true"] * n_true_rules
    apps = ["productpage", "details", "reviews", "ratings"]
    versions = ["v1", "v2", "v3"]
    users = ["cluster.local/ns/default/sa/bookinfo-productpage", "cluster.local/ns/default/sa/bookinfo-reviews",
             "tcp-test-user", "alice", "bob"]
    header_keys = ["x-user", "clnt", "user-agent", "accept", "x-request-id", "x-b3-traceid", "x-b3-spanid",
                   "cookie", "host", "x-forwarded-for", "x-envoy-internal", "content-type", "authorization",
                   "x-custom", "referer"]
    bags = []
    for i in range(n_bags):
        b = {}
        da, dv = apps[rng.integers(4)], versions[rng.integers(3)]
        sa, sv = apps[rng.integers(4)], versions[rng.integers(3)]
        svc = ["foo", "bar", da][rng.integers(3)]
        b["destination.service"] = "%s.default.svc.cluster.local" % svc
        b["destination.labels"] = {"app": da, "version": dv}
        b["source.labels"] = {"app": sa, "version": sv}
        b["source.user"] = users[rng.integers(len(users))]
        hdr = {}
        for k in header_keys:
            if rng.random() < 0.6:
                hdr[k] = ["", "abc", "jason", "xyz", "1"][rng.integers(5)]
        b["request.headers"] = hdr
        if rng.random() < 0.05:
            b["source.ip"] = _ip4(10, 11, 12, 13)
        else:
            b["source.ip"] = _ip4(10, 0, int(rng.integers(256)), int(rng.integers(256)))
        b["context.protocol"] = "tcp" if rng.random() < 0.2 else "http"
        for k in list(b):
            if rng.random() < 0.05:
                del b[k]
        bags.append(b)
    return TESTDATA_MANIFEST, rules, BagBatch.from_bags(bags, names=sorted(
        ["destination.service", "destination.labels", "source.labels", "source.user", "request.headers",
         "source.ip", "context.protocol"]))


def c2_rules(n_rules=1000, seed=2, n_services=256):
    rng = np.random.default_rng(seed)
    ips = rng.integers(0, 256, size=(n_rules, 3))
    rules = []
    for i in range(n_rules):
        a, b, c = (int(x) for x in ips[i])
        rules.append('destination.service == "svc%d.ns%d.svc.cluster.local" && request.path.startsWith("/api/v%d/r%d")'
                     ' && source.ip != ip("10.%d.%d.%d")' % (i % n_services, (i % n_services) % 8, i % 7, i % 97, a, b, c))
    return rules, ips


def c2_workload(n_rules=1000, n_requests=65536, seed=2, n_services=256, p_missing_path=0.01, p_missing_ip=0.005,
                shard=None):
    """C2: ==/startsWith/ip() rules, Zipf(1.1) services.  Returns (manifest, rules, BagBatch).
    shard=(lo, hi): requests [lo, hi) of the n_requests-request batch (every per-request draw is made
    for the whole batch, so the shards of one seed partition that batch exactly)."""
    rules, ips = c2_rules(n_rules, seed, n_services)
    rng = np.random.default_rng(seed + 1000)
    n = n_requests
    lo, hi = shard if shard is not None else (0, n)
    ranks = np.arange(1, n_services + 1, dtype=np.float64)
    p = ranks ** -1.1
    p /= p.sum()
    svc = rng.choice(n_services, size=n, p=p)
    # request paths: half follow one of the service's own rules' prefixes
    rules_per_svc = max(1, (n_rules + n_services - 1) // n_services)
    follow = rng.random(n) < 0.5
    j = rng.integers(0, rules_per_svc, size=n)
    rule_i = svc + n_services * j
    rule_i = np.where(rule_i < n_rules, rule_i, svc % max(n_rules, 1))
    pv = np.where(follow, rule_i % 7, rng.integers(0, 7, size=n))
    pr = np.where(follow, rule_i % 97, rng.integers(0, 97, size=n))
    tail = rng.integers(0, 4096, size=n)
    path_missing = rng.random(n) < p_missing_path
    # source.ip: 4-byte addresses in 10.0.0.0/8; 5% equal to one of the service's rules' ip
    hit = rng.random(n) < 0.05
    a = rng.integers(0, 256, size=n)
    b = rng.integers(0, 256, size=n)
    c = rng.integers(0, 256, size=n)
    ip_missing = rng.random(n) < p_missing_ip
    svc, rule_i, pv, pr, tail, path_missing = (x[lo:hi] for x in (svc, rule_i, pv, pr, tail, path_missing))
    hit, a, b, c, ip_missing = (x[lo:hi] for x in (hit, a, b, c, ip_missing))
    n = hi - lo
    strings = [b"svc%d.ns%d.svc.cluster.local" % (s, s % 8) for s in range(n_services)]
    dest_vals = svc.astype(np.uint64)
    base = len(strings)
    path_keys = (pv * 97 + pr) * 4096 + tail
    uniq, inv = np.unique(path_keys, return_inverse=True)
    for k in uniq:
        k = int(k)
        t = k % 4096
        q = k // 4096
        strings.append(b"/api/v%d/r%d/item%d" % (q // 97, q % 97, t))
    path_vals = (base + inv).astype(np.uint64)
    path_kinds = np.where(path_missing, ABSENT, STRING).astype(np.uint8)
    ri = np.where(rule_i < n_rules, rule_i, 0)
    a = np.where(hit, ips[ri, 0], a)
    b = np.where(hit, ips[ri, 1], b)
    c = np.where(hit, ips[ri, 2], c)
    ip_keys = (a * 256 + b) * 256 + c
    iuniq, iinv = np.unique(ip_keys, return_inverse=True)
    ibase = len(strings)
    for k in iuniq:
        k = int(k)
        strings.append(bytes([10, (k >> 16) & 255, (k >> 8) & 255, k & 255]))
    ip_vals = (ibase + iinv).astype(np.uint64)
    ip_kinds = np.where(ip_missing, ABSENT, BYTES).astype(np.uint8)
    cols = {
        "destination.service": (np.full(n, STRING, dtype=np.uint8), dest_vals),
        "request.path": (path_kinds, path_vals),
        "source.ip": (ip_kinds, ip_vals),
    }
    return TESTDATA_MANIFEST, rules, BagBatch.from_columns(n, cols, strings)


# ----------------------------------------------------------------------------------- fuzzing
_STR_VALS = ["", "a", "abc", "abcd", "foo", "bar", "st.*", "str1", "1.2.3.4", "10.0.0.1", "::1", "(x", "a+b",
             "2015-01-02T15:04:35Z", "2015-01-02T15:04:35+01:00", "*", "a*", "*c", "19ms", "x-user"]
_KEYS = ["a", "b", "c", "foo", "x-user"]
_REGEXES = ["^a", "b.*c", "^(abc|foo)$", "[0-9]+", "\\d\\.\\d", "(?i)ABC", "st.*", "^$", "x*", "\\bfoo\\b"]


class _Fuzz:
    def __init__(self, rng):
        self.r = rng

    def pick(self, xs):
        return xs[int(self.r.integers(len(xs)))]

    def slit(self):
        return '"%s"' % self.pick(_STR_VALS)

    def sexpr(self, d):
        r = self.r.random()
        if d <= 0 or r < 0.35:
            return self.pick(["as", "bs", self.slit()])
        if r < 0.55:
            return '%s[%s]' % (self.pick(["ar", "br", "sm"]), self.pick(['"%s"' % self.pick(_KEYS), "as"]))
        if r < 0.75:
            return '(%s | %s)' % (self.sexpr(d - 1), self.sexpr(d - 1))
        return '(%s | %s)["%s"]' % (self.pick(["ar", "br"]), self.pick(["ar", "br", "sm"]), self.pick(_KEYS))

    def atom(self, d):
        r = self.r.random()
        if r < 0.2:
            return "%s == %s" % (self.sexpr(d), self.sexpr(d))
        if r < 0.3:
            return "%s != %s" % (self.sexpr(d), self.slit())
        if r < 0.4:
            return "%s == %d" % (self.pick(["ai", "bi", "(ai | bi)", "(ai | 7)"]), int(self.r.integers(-2, 5)))
        if r < 0.45:
            return "ai == bi"
        if r < 0.5:
            return "%s == %s" % (self.pick(["ad", "bd", "(ad | 2.5)"]), self.pick(["1.5", "2.5", "0.0", "bd"]))
        if r < 0.58:
            return self.pick(["ab", "bb", "b1", "(ab | bb)", "(ab | true)", "ab == bb", "b1 != false"])
        if r < 0.68:
            fn = self.pick(["startsWith", "endsWith"])
            return "%s.%s(%s)" % (self.pick(["as", "bs", self.slit()]), fn, self.sexpr(d))
        if r < 0.74:
            return "match(%s, %s)" % (self.sexpr(d), self.pick(['"a*"', '"*c"', '"abc"', '"*"', "bs"]))
        if r < 0.82:
            return "%s %s %s" % (self.pick(["aip", "bip", "(aip | bip)"]), self.pick(["==", "!="]),
                                 self.pick(['ip("1.2.3.4")', 'ip("10.0.0.1")', "bip", "ip(as)", 'ip("bad")',
                                            'ip(ar["a"])', 'ip("::ffff:1.2.3.4")']))
        if r < 0.88:
            return "%s == %s" % (self.pick(["at", "t1", "(at | bt)"]),
                                 self.pick(['timestamp("2015-01-02T15:04:35Z")', "t2", "timestamp(as)",
                                            'timestamp("nope")']))
        if r < 0.92:
            return "%s == %s" % (self.pick(["adur", "(adur | bdur)"]), self.pick(['"19ms"', "bdur", '"0"']))
        if r < 0.96:
            return self.pick(['"%s".matches(%s)' % (self.pick(_REGEXES), self.sexpr(d)), "as.matches(bs)",
                              'bs.matches("abc")', '"(bad".matches(as)'])
        return self.pick(["true", "false", "TRUE", "ai == true", "as.foo()", "ai = 2", "x == 2", "ar == br"])

    def expr(self, d):
        r = self.r.random()
        if d <= 0 or r < 0.45:
            return self.atom(d)
        if r < 0.7:
            return "%s && %s" % (self.expr(d - 1), self.expr(d - 1))
        if r < 0.9:
            return "%s || %s" % (self.expr(d - 1), self.expr(d - 1))
        return "(%s)" % self.expr(d - 1)


def fuzz_rules(n, seed=7, depth=3):
    f = _Fuzz(np.random.default_rng(seed))
    return [f.expr(depth) for _ in range(n)]


def hard_fuzz_rules(n, seed=13):
    """Rules at the reference VM's limits (interpreter.go:39-44): long `||` / `&&` chains whose
    resolves and pushes reach heap slot 63 ("heap overflow", interpreterRun.go:171-172), nested
    chains whose paths merge with different heap counts, `ip()` returns that take slot 63 without the
    check so the next push is Go's index panic, `|` chains of comparisons that leave a value behind
    each (up to and past the 64-word stack: "stack overflow"), right-nested comparisons with more
    live values than the hot kernels' 8 registers (the deep kernels), and `matches` patterns
    computed at run time (map values, `|` fallbacks, run-time map keys)."""
    rng = np.random.default_rng(seed)
    f = _Fuzz(rng)
    vals = [v for v in _STR_VALS if v not in ("19ms",)]  # (a duration literal: type error)
    atoms = [lambda: 'as == "%s"' % f.pick(vals), lambda: 'bs != "%s"' % f.pick(vals),
             lambda: 'ar["%s"] == "%s"' % (f.pick(_KEYS), f.pick(vals)),
             lambda: 'as.startsWith("%s")' % f.pick(["a", "ab", "st", ""]), lambda: "ai == %d" % int(rng.integers(0, 5)),
             lambda: '"%s".matches(bs)' % f.pick(["^a", "b.*c", "^$"])]
    pats = ['ar["%s"]' % k for k in _KEYS] + ["as", "bs", 'sm["a"]', "ar[as]", "(ar | br)[\"a\"]"]

    # chain links that rarely decide the chain (false under ||, true under &&), so evaluations run
    # deep into it; a few random atoms in between
    quiet = {"||": [lambda: 'as == "zz%d"' % int(rng.integers(100)), lambda: 'ar["%s"] == "zz"' % f.pick(_KEYS),
                    lambda: "ai == 99", lambda: 'bs.startsWith("zz")', lambda: '"^zz".matches(as)'],
             "&&": [lambda: 'as != "zz%d"' % int(rng.integers(100)), lambda: 'ar["%s"] != "zz"' % f.pick(_KEYS),
                    lambda: "ai != 99", lambda: 'bs.endsWith("zz") == false']}

    def chain(k, op):
        return (" %s " % op).join(f.pick(atoms)() if rng.random() < 0.05 else f.pick(quiet[op])()
                                  for _ in range(k))

    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.2:  # one chain at depth 0
            out.append(chain(int(rng.integers(40, 90)), f.pick(["||", "&&"])))
        elif r < 0.35:  # chains nested under && / || (merges with different heap counts)
            out.append("(%s) && (%s)" % (chain(int(rng.integers(20, 50)), "||"), chain(int(rng.integers(10, 40)), "||")))
        elif r < 0.45:  # slot 63 taken by an ip() return, then a checked push: index panic
            k = int(rng.integers(58, 64))
            out.append(chain(k, "||") + ' || ip(%s) == ip("%s") || %s' % (f.pick(["as", '"1.2.3.4"', 'ar["a"]']),
                                                                        f.pick(["1.2.3.4", "10.0.0.1"]), f.pick(atoms)()))
        elif r < 0.6:  # `|` garbage: each comparison leaves a bool behind
            k = int(rng.integers(3, 80))
            out.append(" | ".join(f.pick(["(ai == %d)" % int(rng.integers(0, 4)), "(ab == bb)", "(ad == 1.5)",
                                          "(bi == ai)", '(as == "zz")', '(ar["a"] == "b")']) for _ in range(k)))
        elif r < 0.75:  # right-nested comparisons: up to 70 values live
            k = int(rng.integers(5, 72))
            e = f.pick(["ab", "bb", "true"])
            for _ in range(k):
                e = "%s == (%s)" % (f.pick(["ab", "bb", "b1", "(ab | bb)"]), e)
            out.append(e)
        else:  # run-time patterns
            p = f.pick(pats)
            fb = f.pick(['"^a"', '"(x"', '"st.*"', "as", '"%s"' % f.pick(_REGEXES).replace("\\", "\\\\")])
            form = rng.random()
            if form < 0.4:
                out.append("(%s | %s).matches(%s)" % (p, fb, f.pick(["as", "bs", 'ar["a"]'])))
            elif form < 0.7:
                out.append("(%s | %s | %s).matches(bs) && %s" % (p, f.pick(pats), fb, f.pick(atoms)()))
            else:
                out.append("%s || (%s | %s).matches(as)" % (f.pick(atoms)(), p, fb))
    return out


def guarded_fuzz_rules(n, seed=11, depth=2, random_tail=True):
    """Rules whose programs start with a leading atom (guard) -- `attr == K`, `attr != K`,
    `map["k"] == K` -- joined by &&, || or alone to a continuation that is either random or one of a
    few constant-varying shapes (so continuation templates are shared).  Columns, want classes,
    negations and modes mix inside every 32-rule group."""
    rng = np.random.default_rng(seed)
    f = _Fuzz(rng)
    guards = [lambda: 'as == "%s"' % f.pick(_STR_VALS),
              lambda: 'bs != "%s"' % f.pick(_STR_VALS),
              lambda: 'ar["%s"] == "%s"' % (f.pick(_KEYS), f.pick(_STR_VALS)),
              lambda: 'sm["%s"] != "%s"' % (f.pick(_KEYS), f.pick(_STR_VALS)),
              lambda: "ai == %d" % int(rng.integers(0, 5)),
              lambda: "ab == %s" % f.pick(["true", "false"]),
              lambda: "ad == %s" % f.pick(["1.5", "2.5", "0.0"]),
              lambda: 'as.startsWith("%s")' % f.pick(["", "a", "ab", "abc", "st", "1.2", "x"]),
              lambda: 'bs.startsWith("%s") == false' % f.pick(["a", "ab"]),
              lambda: '"^%s".matches(bs)' % f.pick(["a", "ab", "st", "str", "a[bc]", "1.2"]),
              lambda: '"^%s".matches(ar["%s"])' % (f.pick(["a", "fo", "ba"]), f.pick(_KEYS))]
    shapes = [lambda: '%s.startsWith("%s") && aip != ip("%s")' % (f.pick(["as", "bs"]), f.pick(["a", "ab", "st", ""]),
                                                                   f.pick(["1.2.3.4", "10.0.0.1"])),
              lambda: 'br["%s"] == "%s"' % (f.pick(_KEYS), f.pick(_STR_VALS)),
              lambda: 'match(bs, "%s") || bi == %d' % (f.pick(["a*", "*c", "abc", "*"]), int(rng.integers(0, 5))),
              lambda: f.expr(depth)]
    if not random_tail:
        shapes = shapes[:3]
    out = []
    for _ in range(n):
        g = f.pick(guards)()
        r = rng.random()
        if r < 0.1:
            out.append(g)
        elif r < 0.75:
            out.append("%s && %s" % (g, f.pick(shapes)()))
        else:
            out.append("%s || %s" % (g, f.pick(shapes)()))
    return out


def fuzz_bags(n, seed=8, p_missing=0.25, p_wrong=0.05):
    rng = np.random.default_rng(seed)
    f = _Fuzz(rng)
    bags = []
    for _ in range(n):
        b = {}
        for name, vt in DEFAULT_TEST_MANIFEST.items():
            if rng.random() < p_missing:
                continue
            wrong = rng.random() < p_wrong
            if wrong:
                b[name] = f.pick(["str", GoInt64(3), True, GoOther("20"), {"a": "b"}, GoFloat64(1.5), b"\x01"])
                continue
            if vt == "STRING":
                b[name] = f.pick(_STR_VALS)
            elif vt == "INT64":
                b[name] = GoInt64(int(rng.integers(-2, 5))) if rng.random() < 0.9 else GoDuration(3)
            elif vt == "DOUBLE":
                b[name] = GoFloat64(f.pick([1.5, 2.5, 0.0, -0.0]))
            elif vt == "BOOL":
                b[name] = bool(rng.random() < 0.5)
            elif vt == "DURATION":
                b[name] = GoDuration(f.pick([19_000_000, 20_000_000, 0]))
            elif vt == "TIMESTAMP":
                b[name] = GoTime(f.pick([1420211075, 1420211074, 1420207475]), 0)
            elif vt == "IP_ADDRESS":
                b[name] = f.pick([bytes([1, 2, 3, 4]), bytes([10, 0, 0, 1]),
                                  bytes(10) + b"\xff\xff" + bytes([1, 2, 3, 4]), bytes(15) + b"\x01"])
            elif vt == "STRING_MAP":
                m = {}
                for k in _KEYS:
                    if rng.random() < 0.5:
                        m[k] = f.pick(_STR_VALS)
                b[name] = m
        bags.append(b)
    return bags


# ----------------------------------------------------------------------------------- resolver
RESOLVER_NAMESPACES = ["istio-system", "default", "ns1", "ns2", "bookinfo"]


def resolver_workload(n_rules=600, n_requests=2000, seed=21):
    """Rules grouped by namespace (contiguous, resolution order) with random variety masks (4
    varieties), TCP flags and some empty matches; requests whose `destination.service` names one of
    the namespaces, an unknown one, none (no dot), is missing or is not a string, and whose
    `context.protocol` is tcp / http / missing / not a string.
    Returns (manifest, rules, conf, batch) with conf = dict(rule_ns, variety_mask, is_tcp,
    empty_match, identity_attr, default_ns)."""
    rng = np.random.default_rng(seed)
    manifest = dict(DEFAULT_TEST_MANIFEST)
    manifest["destination.service"] = "STRING"
    manifest["context.protocol"] = "STRING"
    body = guarded_fuzz_rules(n_rules, seed=seed + 1, random_tail=False)
    counts = rng.multinomial(n_rules, [0.4, 0.2, 0.15, 0.15, 0.1])
    rule_ns = [ns for ns, c in zip(RESOLVER_NAMESPACES, counts) for _ in range(c)]
    empty = rng.random(n_rules) < 0.05
    # "19ms" is a DURATION literal (expr.go:143-146): keep it out so most rules type-check, then make
    # two rules of ns2 always-error (type error) so that namespace's requests fail
    rules = ["" if e else r.replace('"19ms"', '"abc"') for e, r in zip(empty, body)]
    ns2 = [i for i, ns in enumerate(rule_ns) if ns == "ns2" and not empty[i]]
    for i in ns2[:2]:
        rules[i] = 'as == "19ms"'
    conf = dict(rule_ns=rule_ns,
                variety_mask=[int(x) for x in rng.integers(0, 16, size=n_rules)],
                is_tcp=[int(x) for x in (rng.random(n_rules) < 0.2)],
                empty_match=[int(x) for x in empty],
                identity_attr="destination.service", default_ns="istio-system")
    bags = fuzz_bags(n_requests, seed=seed + 2, p_missing=0.0005, p_wrong=0.0002)
    f = _Fuzz(rng)
    for b in bags:
        r = rng.random()
        if r < 0.05:
            b.pop("destination.service", None)
        elif r < 0.08:
            b["destination.service"] = GoInt64(7)
        elif r < 0.12:
            b["destination.service"] = "nodots"
        elif r < 0.2:
            b["destination.service"] = "svc.unknown.svc.cluster.local"
        else:
            b["destination.service"] = "svc%d.%s.svc.cluster.local" % (rng.integers(0, 9), f.pick(RESOLVER_NAMESPACES))
        r = rng.random()
        if r < 0.25:
            b["context.protocol"] = "tcp"
        elif r < 0.8:
            b["context.protocol"] = "http"
        elif r < 0.85:
            b["context.protocol"] = GoInt64(1)
    names = list(manifest)
    return manifest, rules, conf, BagBatch.from_bags(bags, names=names)


# ----------------------------------------------------------------------------------- lists (C3)
def c3_ip_list(n_entries=100_000, n_lookups=1_000_000, seed=3, p_v6=0.1, hit_rate=0.5):
    """C3 CIDR list: IPv4 /8../32 (uniform prefix) and 10% IPv6 /32../128 entries (some without a
    prefix length -> "/32" appended, as ipList.addEntry does, even for IPv6); lookups are address
    strings, half drawn inside entries, plus a few invalid symbols.  Returns (entries, symbols)."""
    rng = np.random.default_rng(seed)
    entries, nets = [], []
    for _ in range(n_entries):
        if rng.random() < p_v6:
            bits = int(rng.integers(32, 129))
            words = rng.integers(0, 1 << 16, size=8)
            words[0] = 0x2001
            a = ":".join("%x" % w for w in words)
            entries.append(a if rng.random() < 0.05 else "%s/%d" % (a, bits))
            nets.append(("6", words, bits))
        else:
            bits = int(rng.integers(8, 33))
            q = rng.integers(0, 256, size=4)
            a = "%d.%d.%d.%d" % tuple(q)
            entries.append(a if bits == 32 and rng.random() < 0.5 else "%s/%d" % (a, bits))
            nets.append(("4", q, bits))
    # lookups, drawn column-wise (1M in about a second)
    n = n_lookups
    bad = rng.random(n) < 0.01
    pick = rng.integers(0, n_entries, size=n)
    hit = rng.random(n) < hit_rate
    host = rng.integers(0, 1 << 32, size=n, dtype=np.uint64)
    mapped = rng.random(n) <= 0.02
    rnd6 = rng.integers(0, 1 << 16, size=(n, 8))
    is6 = np.array([k == "6" for k, _, _ in nets])[pick]
    base4 = np.array([int(b[0]) << 24 | int(b[1]) << 16 | int(b[2]) << 8 | int(b[3]) if k == "4" else 0
                      for k, b, _ in nets], dtype=np.uint64)[pick]
    bits = np.array([b for _, _, b in nets], dtype=np.uint64)[pick]
    keep = np.where(bits > 0, (np.uint64(0xFFFFFFFF) << (np.uint64(32) - np.minimum(bits, 32))) & np.uint64(0xFFFFFFFF),
                    np.uint64(0))
    x4 = np.where(hit, (base4 & keep) | (host & ~keep & np.uint64(0xFFFFFFFF)), host)
    syms = []
    for q in range(n):
        if bad[q]:
            syms.append("not-an-ip")
        elif not is6[q]:
            x = int(x4[q])
            v = "%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255)
            syms.append("::ffff:" + v if mapped[q] else v)
        else:
            _, base, b6 = nets[int(pick[q])]
            w = [int(v) for v in base] if hit[q] else [int(v) for v in rnd6[q]]
            if hit[q]:
                for i in range(b6 // 16 + 1, 8):
                    w[i] = int(rnd6[q, i])
            syms.append(":".join("%x" % v for v in w))
    return entries, syms


def c3_string_list(n_entries=100_000, n_lookups=1_000_000, seed=3, hit_rate=0.5):
    """C3 string list: ASCII entries of 8..64 bytes; lookups half hits (some with case changed,
    for the case-insensitive kind), half misses.  Returns (entries, symbols)."""
    rng = np.random.default_rng(seed + 7)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_./", dtype=np.uint8)
    lens = rng.integers(8, 65, size=n_entries)
    entries = [bytes(alpha[rng.integers(0, len(alpha), size=int(n))]).decode() for n in lens]
    idx = rng.integers(0, n_entries, size=n_lookups)
    hit = rng.random(n_lookups) < hit_rate
    syms = []
    for i, h in zip(idx, hit):
        e = entries[int(i)]
        if not h:
            e = e[:-1] + ("#" if e[-1] != "#" else "%")
        elif rng.random() < 0.3:
            e = e.swapcase()
        syms.append(e)
    return entries, syms


def c3_regex_list(n_patterns=10_000, n_lookups=1_000_000, seed=3, hit_rate=0.5, return_hits=False):
    """C3 regex list: patterns `^prefix[a-z0-9]{m,n}(suffix)?$`; lookups half built
    to match a random pattern, half near misses.  Returns (patterns, symbols) (+ a bool array of the
    lookups built to match, with return_hits)."""
    rng = np.random.default_rng(seed + 11)
    letters = "abcdefghijklmnopqrstuvwxyz"
    alnum = letters + "0123456789"

    def word(lo, hi):
        return "".join(letters[int(i)] for i in rng.integers(0, 26, size=int(rng.integers(lo, hi + 1))))
    specs, pats = [], []
    for _ in range(n_patterns):
        pre, suf = word(3, 8), word(2, 5)
        m = int(rng.integers(1, 4))
        n = m + int(rng.integers(0, 6))
        specs.append((pre, m, n, suf))
        pats.append("^%s[a-z0-9]{%d,%d}(%s)?$" % (pre, m, n, suf))
    # lookups, drawn column-wise
    nl = n_lookups
    sel = rng.integers(0, n_patterns, size=nl)
    lo = np.array([sp[1] for sp in specs])[sel]
    hi = np.array([sp[2] for sp in specs])[sel]
    blen = lo + (rng.random(nl) * (hi - lo + 1)).astype(np.int64)
    body = np.frombuffer(alnum.encode(), dtype=np.uint8)[rng.integers(0, 36, size=(nl, 8))].tobytes().decode()
    with_suf = rng.random(nl) < 0.5
    hits = rng.random(nl) < hit_rate
    tail = np.where(rng.random(nl) < 0.5, "-", "X")
    syms = []
    for q in range(nl):
        pre, _, _, suf = specs[int(sel[q])]
        s = pre + body[8 * q:8 * q + int(blen[q])] + (suf if with_suf[q] else "")
        syms.append(s if hits[q] else s + tail[q])  # a miss: outside the class / past the anchor
    return (pats, syms, np.array(hits)) if return_hits else (pats, syms)


# ----------------------------------------------------------------------------------- C4 routes
C4_MANIFEST = {"request.path": "STRING", "request.headers": "STRING_MAP", "destination.service": "STRING"}
_C4_HEADERS = ["x-user", "x-env", "x-canary", "user-agent", "x-region"]


def c4_workload(n_rules=10000, n_requests=1_000_000, seed=4, vocab=512, cont_frac=0.0, paths_only=False, shard=None):
    """C4: Pilot-shaped HTTP route rules in the Mixer language: 60%
    request.path.startsWith("/p..") (Pilot prefix), 20% "^...".matches(request.path) (Pilot regex:
    prefix -> ^QuoteMeta(p).*), 20% request.headers["h"] == "v" or "re".matches(request.headers["h"]).
    Requests: paths of depth 1..6 over a `vocab`-word vocabulary, 3 headers each.
    cont_frac > 0 (tests): that fraction of the prefix rules continue with
    `&& source.ip == ip("10.0.0.K")`, over a source.ip column absent for 30% of the requests -- the
    guard-index kernel then finds true pairs and lookup-error pairs.  paths_only: the header rules'
    share becomes path rules too (a route table matched on paths alone: no value classes).
    shard=(lo, hi): requests [lo, hi) of the n_requests-request batch (drawn whole, then cut).
    Returns (manifest, rules, BagBatch)."""
    rng = np.random.default_rng(seed)
    words = ["w%d" % i for i in range(vocab)]
    vals = ["v%d" % i for i in range(16)]

    def path(depth):
        return "/" + "/".join(words[int(i)] for i in rng.integers(0, vocab, size=depth))
    rules = []
    for i in range(n_rules):
        r = rng.random()
        if paths_only and r >= 0.8:
            r = 0.75 * (r - 0.8) / 0.2  # (prefix and regex rules in their 3:1 proportion)
        p = path(int(rng.integers(1, 4)))
        if r < 0.6:
            if cont_frac and rng.random() < cont_frac:
                rules.append('request.path.startsWith("%s") && source.ip == ip("10.0.0.%d")' % (p, int(rng.integers(0, 4))))
            else:
                rules.append('request.path.startsWith("%s")' % p)
        elif r < 0.8:
            rx = "^" + p + ("(/.*)?$" if rng.random() < 0.5 else "[0-9a-z/]*")
            rules.append('"%s".matches(request.path)' % rx)
        elif r < 0.9:
            rules.append('request.headers["%s"] == "%s"' % (_C4_HEADERS[int(rng.integers(0, 5))],
                                                          vals[int(rng.integers(0, 16))]))
        else:
            rules.append('"^v(1|%d)[0-9]?$".matches(request.headers["%s"])' % (int(rng.integers(2, 9)),
                                                                             _C4_HEADERS[int(rng.integers(0, 5))]))
    # requests, drawn column-wise (1M requests in seconds): path of depth 1..6, the service, 3 of the
    # 5 headers (distinct names, in draw order) with values v0..v15
    n = n_requests
    lo, hi = shard if shard is not None else (0, n)
    depth = rng.integers(1, 7, size=n)[lo:hi]
    w = rng.integers(0, vocab, size=(n, 6))[lo:hi]
    hdr = np.argsort(rng.random((n, 5)), axis=1)[lo:hi, :3]
    hval = rng.integers(0, 16, size=(n, 3))[lo:hi]
    n_all, n = n, hi - lo
    strings = [h.encode() for h in _C4_HEADERS] + [v.encode() for v in vals] + [b"svc.default.svc.cluster.local"]
    svc_sid = len(strings) - 1
    paths = {}
    path_vals = np.empty(n, dtype=np.uint64)
    wl = w.tolist()
    for q, d in enumerate(depth.tolist()):
        p = "/" + "/".join(words[i] for i in wl[q][:d])
        sid = paths.get(p)
        if sid is None:
            sid = paths[p] = len(strings)
            strings.append(p.encode())
        path_vals[q] = sid
    moff = np.arange(0, 3 * n + 1, 3, dtype=np.uint64)
    mkeys = hdr.reshape(-1).astype(np.uint32)                    # header name sids 0..4
    mvals = (5 + hval).reshape(-1).astype(np.uint32)             # value sids 5..20
    cols = {"request.path": (np.full(n, STRING, dtype=np.uint8), path_vals),
            "request.headers": (np.full(n, STRING_MAP, dtype=np.uint8), np.arange(n, dtype=np.uint64)),
            "destination.service": (np.full(n, STRING, dtype=np.uint8), np.full(n, svc_sid, dtype=np.uint64))}
    manifest = C4_MANIFEST
    if cont_frac:
        manifest = dict(C4_MANIFEST, **{"source.ip": "IP_ADDRESS"})
        ip0 = len(strings)
        strings.extend(bytes([10, 0, 0, k]) for k in range(4))
        cols["source.ip"] = (np.where(rng.random(n_all)[lo:hi] < 0.3, ABSENT, BYTES).astype(np.uint8),
                             (ip0 + rng.integers(0, 4, size=n_all)[lo:hi]).astype(np.uint64))
    return manifest, rules, BagBatch.from_columns(n, cols, strings, maps=(moff, mkeys, mvals))


# ----------------------------------------------------------------------------------- memquota (C5)
def quota_key_weights(n_keys=1024):
    """C5's key distribution: Zipf(1.05) over the key ids (the expected share of each key)."""
    p = np.arange(1, n_keys + 1, dtype=np.float64) ** -1.05
    return p / p.sum()


def quota_workload(n_keys=1024, n_requests=1_000_000, seed=5, p_free=0.1, p_zero=0.02, p_be=0.5, rank=0, world=1,
                   return_index=False):
    """C5 memquota deltas: K quota keys (a third non-expiring cells, the rest 1 s / 60 s rolling
    windows) with limits 50..5000, requests in arrival order (Zipf keys, amounts 1..20, some frees
    and zero amounts, best effort half the time).  Returns (max_amount, valid_ns, keys, amounts, be).

    Multi-GPU (world > 1): ONE global arrival stream of n_requests * world requests is drawn and
    routed by key owner (dist.key_owners over the keys' expected frequencies, quota_key_weights), as
    an upstream router would; rank `rank` gets the requests of the keys it owns, in global arrival
    order -- so the per-key sequences are the global ones and the union over ranks is exactly the
    single-process workload.  return_index adds the positions of the rank's requests in the global
    stream."""
    rng = np.random.default_rng(seed)
    max_amount = rng.integers(50, 5001, size=n_keys).astype(np.int64)
    valid = np.choose(rng.integers(0, 3, size=n_keys), [0, 10**9, 60 * 10**9]).astype(np.int64)
    p = quota_key_weights(n_keys)
    total = n_requests * world
    keys = rng.choice(n_keys, size=total, p=p).astype(np.uint32)
    amounts = rng.integers(1, 21, size=total).astype(np.int64)
    r = rng.random(total)
    amounts = np.where(r < p_free, -amounts, amounts)
    amounts = np.where(r > 1 - p_zero, 0, amounts)
    be = (rng.random(total) < p_be).astype(np.uint8)
    idx = np.arange(total)
    if world > 1:
        from istio_amd import dist as D
        idx = np.nonzero(D.key_owners(p, world)[keys] == rank)[0]
        keys, amounts, be = keys[idx], amounts[idx], be[idx]
    out = (max_amount, valid, keys, amounts, be)
    return out + (idx,) if return_index else out


# pieces of case-insensitive list symbols beyond ASCII (Go 1.9 strings.ToUpper, goupper.h): case
# pairs, runes with no simple uppercase (ß, ŉ, Georgian in 9.0), runes whose capital is ASCII (ı, ſ),
# titlecase digraphs, Greek with iota subscripts, astral scripts, and invalid UTF-8 bytes
CI_PIECES = ["a", "B", "z", "é", "É", "ß", "ı", "I", "İ", "ſ", "s", "S", "ǅ", "ǆ", "Ǆ", "ᾀ", "ᾈ", "ω", "Ω",
             "σ", "ς", "Σ", "ა", "ꭓ", "Ꭓ", "\U0001e922", "\U0001e900", "\udcff", "\udcc3", "\udca9", "\udce2\udc82",
             "0", "-", "ÿ", "Ÿ", "µ", "Μ"]


def ci_unicode_list(n_entries=3000, n_lookups=20000, seed=41):
    """Case-insensitive list entries and lookups mixing ASCII, non-ASCII and invalid UTF-8 (str with
    surrogate escapes for raw bytes)."""
    rng = np.random.default_rng(seed)

    def word(lo, hi):
        return "".join(CI_PIECES[i] for i in rng.integers(0, len(CI_PIECES), int(rng.integers(lo, hi))))
    return [word(1, 5) for _ in range(n_entries)], [word(0, 5) for _ in range(n_lookups)]


def split_batch(batch, n_members):
    """The contiguous shards of one batch (dist.shard_bounds / mxp_group_shard_bounds): member k's
    requests as a BagBatch whose columns are views into the batch's and whose string / time / map
    tables are the batch's own."""
    from istio_amd.bags import BagBatch
    from istio_amd.dist import shard_bounds
    out = []
    for k in range(n_members):
        lo, hi = shard_bounds(batch.n, k, n_members)
        out.append(BagBatch(hi - lo, batch.names, [c[lo:hi] for c in batch.kinds], [v[lo:hi] for v in batch.values],
                            batch.str_blob, batch.str_offsets, batch.time_sec, batch.time_nsec, batch.map_offsets,
                            batch.map_keys, batch.map_values))
    return out
