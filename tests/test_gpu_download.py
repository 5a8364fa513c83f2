"""Downloads into caller memory (engine.cpp download / download_all): pinned memory is written by
the shader copy (mxp_d2h_copy_kernel: 16-byte words when the two sides share their alignment,
bytewise otherwise), pageable memory through the pinned bounce pair, and MXP_D2H_DMA=1 keeps the
copy engine.  Every path must hand back the same Resolve outputs as pageable numpy arrays."""
import ctypes

import numpy as np
import pytest

from istio_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mxp(libmxp):
    import istio_amd.engine as mxp
    return mxp


def _engine(mxp, manifest, rules):
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    R = len(rules)
    # the default namespace, then contiguous blocks of the workload's namespaces ns0..ns7 (requests
    # select different lists); every rule of variety 0
    rest = R - R // 2
    ns = ["istio-system"] * (R // 2) + ["ns%d" % (8 * i // rest) for i in range(rest)]
    eng.set_resolver("destination.service", "istio-system", ns, np.ones(R, dtype=np.uint32),
                     np.zeros(R, dtype=np.uint8), np.zeros(R, dtype=np.uint8))
    return eng


@pytest.fixture(scope="module")
def case(mxp):
    manifest, rules, batch = W.c2_workload(n_rules=1200, n_requests=300_000, seed=21)
    return manifest, rules, batch


def test_pinned_outputs_equal_pageable(mxp, case):
    manifest, rules, batch = case
    eng = _engine(mxp, manifest, rules)
    want = [x.copy() for x in eng.resolve_arrays(batch, 0, ids16=True)]
    for _ in range(2):  # (the second call reuses the arena)
        got = eng.resolve_arrays(batch, 0, ids16=True, pinned=True)
        for a, b in zip(want, got):
            assert np.array_equal(a, b)
    pb, arena = mxp.pinned_batch(batch)
    got = eng.resolve_arrays(pb, 0, ids16=True, pinned=True)
    for a, b in zip(want, got):
        assert np.array_equal(a, b)
    arena.free()
    eng.close()


@pytest.mark.parametrize("dma", ["0", "1"])
def test_misaligned_pinned_outputs(mxp, case, monkeypatch, dma):
    """Outputs at odd byte offsets of a pinned arena (the shader copy's bytewise path, and its
    16-byte path with a head and a tail), against pageable outputs."""
    monkeypatch.setenv("MXP_D2H_DMA", dma)
    manifest, rules, batch = case
    eng = _engine(mxp, manifest, rules)
    st0, er0, off0, sel0 = (x.copy() for x in eng.resolve_arrays(batch, 0))
    n, total = batch.n, int(off0[-1])
    assert total > 1000
    arena = mxp.PinnedArena(n * 13 + total * 4 + 4096)
    base = arena.p.value
    # status at +3, err_rule at +16k+5 (u32 at an odd address), sel_off at +8 mod 16, sel at +1
    o_st = 3
    o_er = ((o_st + n + 63) & ~63) + 5
    o_off = ((o_er + 4 * n + 63) & ~63) + 8
    o_sel = ((o_off + 8 * (n + 1) + 63) & ~63) + 1
    assert o_sel + 4 * total <= arena.size
    ctypes.memset(base, 0xAB, arena.size)
    rc = eng.lib.mxp_resolve_batch(eng.h, ctypes.byref(batch.c_struct()), 0, base + o_st, base + o_er, base + o_off,
                                   base + o_sel, total)
    eng._check(rc, "mxp_resolve_batch")
    raw = np.frombuffer((ctypes.c_uint8 * arena.size).from_address(base), dtype=np.uint8)
    st = raw[o_st:o_st + n]
    er = raw[o_er:o_er + 4 * n].copy().view(np.uint32)
    off = raw[o_off:o_off + 8 * (n + 1)].copy().view(np.uint64)
    sel = raw[o_sel:o_sel + 4 * total].copy().view(np.uint32)
    assert np.array_equal(st, st0) and np.array_equal(er, er0) and np.array_equal(off, off0)
    assert np.array_equal(sel, sel0)
    assert raw[o_st - 1] == 0xAB and raw[o_st + n] == 0xAB and raw[o_sel + 4 * total] == 0xAB  # (no spill)
    arena.free()
    eng.close()


def test_large_pageable_download(mxp, case):
    """Bitmaps past the bounce buffers' 32 MiB (several chunks into pageable numpy memory) equal
    the same evaluation copied out of device memory by torch."""
    import torch
    manifest, rules, batch = case
    eng = mxp.Engine(0)
    eng.set_vocabulary(manifest)
    assert (eng.compile(rules) == 0).all()
    m, e = eng.eval_batch(batch)
    assert m.nbytes > (32 << 20)
    db = eng.upload(batch)
    Wd = (len(rules) + 31) // 32
    dm = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda")
    de = torch.empty((Wd, batch.n), dtype=torch.int32, device="cuda")
    db.eval(dm.data_ptr(), de.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(dm.cpu().numpy().view(np.uint32), m)
    assert np.array_equal(de.cpu().numpy().view(np.uint32), e)
    db.free()
    eng.close()
