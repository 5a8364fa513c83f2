"""The device packer (pack_device.cpp / pack.hip: interning, column gather, ip() / timestamp()
pre-tables and value-class sizing on the GPU) against the host packer (MXP_HOST_PACK=1, engine.cpp
pack_host): identical match / error bitmaps and identical error texts on workloads that carry
strings, byte strings (IP addresses), timestamps, string maps, virtual map[key] columns and run-time
regexp patterns -- and both against the oracle through the parity tests, which now pack on the
device by default."""
import numpy as np
import pytest

from istio_amd import workloads as W
from istio_amd.bags import BagBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _run(mxp, monkeypatch, host, manifest, rules, batch, flags="0"):
    monkeypatch.setenv("MXP_HOST_PACK", "1" if host else "0")
    monkeypatch.setenv("MXP_DEBUG_FLAGS", flags)
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    m, e = eng.eval_batch(batch)
    codes = mxp.bits_to_codes(m, e, len(rules))
    errs = np.argwhere(codes == 2)
    rng = np.random.default_rng(3)
    if len(errs) > 400:
        errs = errs[rng.choice(len(errs), 400, replace=False)]
    texts = [(int(q), int(r), eng.pair_error(int(q), int(r))) for q, r in errs]
    return m, e, texts


@pytest.mark.parametrize("wl,flags", [("fuzz", "0"), ("fuzz", "262144"), ("c1", "0"), ("c2", "0"), ("c4", "0"),
                                      ("resolver", "0")])
def test_device_pack_matches_host_pack(mxp, monkeypatch, wl, flags):
    if wl == "fuzz":
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.fuzz_rules(600, seed=91, depth=3)
        batch = BagBatch.from_bags(W.fuzz_bags(4000, seed=92), names=list(manifest))
    elif wl == "c1":
        manifest, rules, batch = W.c1_workload(6000)
    elif wl == "c2":
        manifest, rules, batch = W.c2_workload(n_rules=800, n_requests=20000)
    elif wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=12000, seed=93)
    else:
        manifest, rules, conf, batch = W.resolver_workload(n_rules=300, n_requests=3000, seed=94)
    mh, eh, th = _run(mxp, monkeypatch, True, manifest, rules, batch, flags)
    md, ed, td = _run(mxp, monkeypatch, False, manifest, rules, batch, flags)
    assert np.array_equal(mh, md) and np.array_equal(eh, ed)
    assert th == td
    assert all(t for _, _, t in td)


def test_device_pack_edge_batches(mxp, monkeypatch):
    """Empty batches, a batch without strings, duplicate strings in the batch table, strings equal
    to rule-set constants and absent columns."""
    manifest = {"a": "STRING", "b": "STRING", "t": "TIMESTAMP", "ip": "IP_ADDRESS", "m": "STRING_MAP"}
    rules = ['a == "x"', 'a == b', 'b.startsWith("y")', 'm["k"] == a', 'ip(a) == ip("1.2.3.4")',
             'timestamp(b) == t', '"^x".matches(a)', 'a.matches(b)']
    bags = [{"a": "x", "b": "x"}, {"a": "1.2.3.4", "b": "2015-01-02T15:04:35Z"}, {"m": {"k": "x"}, "a": "x"},
            {"a": "yy", "b": "^y"}, {}, {"a": "", "b": ""}, {"ip": bytes([1, 2, 3, 4]), "a": "1.2.3.4"}]
    for bs in ([], bags[4:5], bags, bags * 50):
        batch = BagBatch.from_bags(bs, names=list(manifest))
        out = [_run(mxp, monkeypatch, host, manifest, rules, batch) for host in (True, False)]
        assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
        assert out[0][2] == out[1][2]


@pytest.mark.parametrize("wl", ["fuzz", "c1", "c4", "resolver"])
def test_narrow_device_pack_matches_host_pack(mxp, monkeypatch, wl):
    """The narrow batch (mxp_batch_upload2: u32 ids and offsets widened on the device, checked as
    u32, the host view widened only for the passes that read it -- run-time regexp patterns among
    them) packs to the same bitmaps as the host packer on the wide batch."""
    from istio_amd.bags import NarrowBatch
    from test_gpu_narrow import _bitmaps
    if wl == "fuzz":
        manifest = W.DEFAULT_TEST_MANIFEST
        rules = W.fuzz_rules(600, seed=95, depth=3)
        batch = BagBatch.from_bags(W.fuzz_bags(4000, seed=96, p_wrong=0.0), names=list(manifest))  # (wrong kinds: no narrow column)
    elif wl == "c1":
        manifest, rules, batch = W.c1_workload(6000)
    elif wl == "c4":
        manifest, rules, batch = W.c4_workload(n_rules=1500, n_requests=12000, seed=97)
    else:
        manifest, rules, conf, batch = W.resolver_workload(n_rules=300, n_requests=3000, seed=98)
    mh, eh, _ = _run(mxp, monkeypatch, True, manifest, rules, batch)
    monkeypatch.setenv("MXP_HOST_PACK", "0")
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    eng.compile(rules)
    nb = NarrowBatch(batch)
    assert nb.narrow.any()
    md, ed = _bitmaps(eng.upload2(nb), batch.n, len(rules))
    assert np.array_equal(mh, md.view(np.uint32)) and np.array_equal(eh, ed.view(np.uint32))
