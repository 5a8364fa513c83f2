"""Host mirror of the reference's evaluator / resolver interfaces over the C-ABI (include/mxp.h).

`Evaluator` mirrors `expr.Evaluator` as implemented by `evaluator.IL`
(mixer/pkg/expr/evaluator.go:25-31, mixer/pkg/il/evaluator/evaluator.go:36-200): `eval` /
`eval_predicate` on an expression text and one bag, `change_vocabulary`.  `Engine` is the batched
form the drop-in actually uses: compile a rule set once, then evaluate whole batches of bags on the
GPU (`eval_batch` -> per-pair match / error bitmaps, `pair_error` -> the reference's error text).

There is no CPU fallback: every evaluation runs the HIP kernels in libmxp.so, and loading fails
loudly when the library (or a GPU) is missing.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from .bags import BagBatch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MXP_LIB") or os.path.join(_HERE, "libmxp.so")  # MXP_LIB: A/B of builds

VALUE_TYPES = {"VALUE_TYPE_UNSPECIFIED": 0, "STRING": 1, "INT64": 2, "DOUBLE": 3, "BOOL": 4, "TIMESTAMP": 5,
               "IP_ADDRESS": 6, "EMAIL_ADDRESS": 7, "URI": 8, "DNS_NAME": 9, "DURATION": 10, "STRING_MAP": 11}

RULE_OK, RULE_PARSE_ERROR, RULE_TYPE_ERROR, RULE_COMPILE_ERROR, RULE_COMPILE_PANIC, RULE_UNSUPPORTED = range(6)
FALSE, TRUE, ERROR, PANIC = 0, 1, 2, 3

# mxp_attr_finder (mxp.h): int32_t (*)(void* ctx, const char* name)
_FINDER = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_char_p)

# every entry point declared in include/mxp.h: name -> (restype, argtypes)
_VP = ctypes.c_void_p
SIGNATURES = {
    "mxp_engine_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_VP)]),
    "mxp_engine_destroy": (None, [_VP]),
    "mxp_last_error": (ctypes.c_char_p, [_VP]),
    "mxp_vocab_set": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32]),
    "mxp_vocab_set_finder": (ctypes.c_int, [_VP, _VP, _VP]),
    "mxp_vocab_name": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_ruleset_compile": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32)]),
    "mxp_rule_error": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_rule_il_text": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_rule_vm_text": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_rule_types": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "mxp_eval_batch": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "mxp_eval_refs": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64]),
    "mxp_string_text": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_wire_decode": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_wire_view": (_VP, [_VP]),
    "mxp_wire_free": (None, [_VP]),
    "mxp_listentry_check": (ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, ctypes.c_uint32, _VP, _VP]),
    "mxp_resolve_refs": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, _VP, _VP, _VP, _VP, ctypes.c_uint64, _VP, _VP,
                                        ctypes.c_uint64]),
    "mxp_eval_values": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "mxp_value_text": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_value_kind": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint64]),
    "mxp_value_decode": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint64, _VP, _VP, ctypes.c_uint32]),
    "mxp_pair_error": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_error_count": (ctypes.c_uint64, [_VP]),
    "mxp_batch_upload": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(_VP)]),
    "mxp_batch_upload_ex": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_batch_wait_copied": (ctypes.c_int, [_VP]),
    "mxp_batch_pack_host": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]),
    "mxp_batch_free": (None, [_VP, _VP]),
    "mxp_batch_eval_device": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "mxp_hits_device": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, _VP, _VP]),
    "mxp_rule_count": (ctypes.c_uint32, [_VP]),
    "mxp_dbatch_requests": (ctypes.c_uint32, [_VP]),
    "mxp_resolver_set": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "mxp_resolve_batch": (ctypes.c_int, [_VP, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "mxp_resolve_batch_ex": (ctypes.c_int, [_VP, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "mxp_list_create": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_list_destroy": (None, [_VP, _VP]),
    "mxp_list_entries": (ctypes.c_uint64, [_VP]),
    "mxp_list_regex_parts": (None, [_VP, ctypes.c_void_p]),
    "mxp_list_regex_dispatch": (None, [_VP, ctypes.c_void_p]),
    "mxp_list_check": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_void_p]),
    "mxp_list_check_device": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "mxp_regex_match_host": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                            ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_quota_create": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(_VP)]),
    "mxp_quota_destroy": (None, [_VP, _VP]),
    "mxp_quota_alloc": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p]),
    "mxp_quota_alloc_device": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    "mxp_batch_eval_device_hits": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    "mxp_batch_eval_device_compact": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    "mxp_set_timing": (ctypes.c_int, [_VP, ctypes.c_int]),
    "mxp_set_pipeline": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32]),
    "mxp_kernel_times": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    "mxp_ruleset_info": (ctypes.c_uint32, [_VP, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "mxp_ruleset_columns": (ctypes.c_uint32, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint32]),
    "mxp_debug_wave_times": (ctypes.c_int, [_VP, _VP, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "mxp_debug_bin": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64)]),
    "mxp_host_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_VP)]),
    "mxp_host_free": (None, [_VP]),
    "mxp_go_to_upper": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, _VP, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64)]),
    # device groups (include/mxp_group.h)
    "mxp_group_create": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_group_destroy": (None, [_VP]),
    "mxp_group_last_error": (ctypes.c_char_p, [_VP]),
    "mxp_group_size": (ctypes.c_uint32, [_VP]),
    "mxp_group_reduce_mode": (ctypes.c_int, [_VP]),
    "mxp_group_engine": (_VP, [_VP, ctypes.c_uint32]),
    "mxp_group_stream": (_VP, [_VP, ctypes.c_uint32]),
    "mxp_group_shard_bounds": (None, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "mxp_group_locate": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]),
    "mxp_group_vocab_set": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int32),
                                           ctypes.c_uint32]),
    "mxp_group_vocab_set_finder": (ctypes.c_int, [_VP, _VP, _VP]),
    "mxp_group_ruleset_compile": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_int32)]),
    "mxp_group_resolver_set": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                              _VP, _VP, _VP, ctypes.c_uint32]),
    "mxp_group_upload": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_group_upload2": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_batch_upload2": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_group_upload_split": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "mxp_group_batch_wait_copied": (ctypes.c_int, [_VP]),
    "mxp_group_batch_free": (None, [_VP, _VP]),
    "mxp_group_batch_requests": (ctypes.c_uint32, [_VP, ctypes.c_uint32]),
    "mxp_group_eval": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32]),
    "mxp_group_download": (ctypes.c_int, [_VP, ctypes.c_uint32, _VP, _VP, _VP]),
    "mxp_group_quota_create": (ctypes.c_int, [_VP, ctypes.c_uint32, _VP, _VP, _VP, ctypes.POINTER(_VP)]),
    "mxp_group_quota_destroy": (None, [_VP, _VP]),
    "mxp_group_quota_upload": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, _VP, _VP, _VP, ctypes.POINTER(_VP)]),
    "mxp_group_quota_eval": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int64]),
    "mxp_group_quota_granted": (ctypes.c_int, [_VP, _VP, _VP]),
    "mxp_group_quota_batch_free": (None, [_VP, _VP]),
    "mxp_group_quota_batch_requests": (ctypes.c_uint32, [_VP, ctypes.c_uint32]),
    "mxp_group_quota_alloc": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, _VP, _VP, _VP, ctypes.c_int64, _VP]),
    "mxp_group_key_owners": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32, _VP]),
    "mxp_group_reduce": (ctypes.c_int, [_VP]),
    "mxp_group_counters": (ctypes.c_int, [_VP, _VP, _VP]),
    "mxp_group_counters_reset": (ctypes.c_int, [_VP]),
    "mxp_group_sync": (ctypes.c_int, [_VP]),
    "mxp_group_resolve_batch": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP,
                                               _VP, _VP, ctypes.c_uint64]),
    "mxp_group_resolve_uploaded": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _VP,
                                                  _VP, _VP, _VP, ctypes.c_uint64]),
    "mxp_resolve_submit": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint32, ctypes.c_uint32, _VP]),
    "mxp_resolve_finish": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64]),
    "mxp_group_resolve_submit": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _VP]),
    "mxp_group_resolve_finish": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64]),
    "mxp_resolve_uploaded": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP, _VP, _VP,
                                            ctypes.c_uint64]),
    "mxp_group_resolve_split": (ctypes.c_int, [_VP, _VP, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP, _VP, _VP,
                                               ctypes.c_uint64]),
    "mxp_group_pair_error": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    "mxp_group_list_create": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, ctypes.c_uint32, _VP, _VP, ctypes.c_uint32,
                                             ctypes.POINTER(_VP)]),
    "mxp_group_list_destroy": (None, [_VP, _VP]),
    "mxp_group_list_member": (_VP, [_VP, ctypes.c_uint32]),
    "mxp_group_list_check": (ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, _VP, ctypes.c_uint32, _VP]),
    "mxp_group_list_check_device": (ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, _VP, _VP, _VP]),
}

_LIB = None


def load_library(path: str = LIB_PATH):
    """Load libmxp.so (built by istio_amd.build); raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(path):
            raise RuntimeError("libmxp.so not built: run `python -m istio_amd.build` (no CPU fallback exists)")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7; load it first so
        # libmxp binds to the same runtime (device pointers and streams are shared with torch).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("MXP_LIB") and not hasattr(lib, name):
                continue  # an older build under A/B (tools/ab_libs.sh): entry points it predates
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _LIB = lib
    return _LIB


class PinnedArena:
    """Page-locked host memory from mxp_host_alloc, handed out as numpy arrays (the arrays of a batch
    a binding packs bags into: DMA to the device at the link's rate).  Freed with the arena."""

    def __init__(self, nbytes: int):
        self.lib = load_library()
        self.p = _VP()
        if self.lib.mxp_host_alloc(max(int(nbytes), 16), ctypes.byref(self.p)) != 0:
            raise MxpError("mxp_host_alloc(%d) failed" % nbytes)
        self.size, self.used = max(int(nbytes), 16), 0

    def empty(self, count: int, dtype) -> np.ndarray:
        """An uninitialised pinned array of `count` elements, 64-byte aligned within the arena."""
        dtype = np.dtype(dtype)
        nb = int(count) * dtype.itemsize
        at = (self.used + 63) & ~63
        if at + nb > self.size:
            raise MxpError("pinned arena full")
        self.used = at + nb
        buf = (ctypes.c_uint8 * max(nb, 1)).from_address(self.p.value + at)
        return np.frombuffer(buf, dtype=dtype, count=int(count))

    def array(self, like: np.ndarray) -> np.ndarray:
        """A pinned copy of `like` (same dtype and shape)."""
        out = self.empty(like.size, like.dtype).reshape(like.shape)
        out[...] = like
        return out

    def free(self):
        if self.p:
            self.lib.mxp_host_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pinned_batch(batch: BagBatch):
    """(a copy of `batch` whose arrays live in pinned memory, the arena that holds them)."""
    arrays = list(batch.kinds) + list(batch.values) + [batch.str_blob, batch.str_offsets, batch.time_sec,
                                                       batch.time_nsec, batch.map_offsets, batch.map_keys,
                                                       batch.map_values]
    arena = PinnedArena(sum(a.nbytes + 64 for a in arrays) + 64)
    nc = len(batch.kinds)
    p = [arena.array(a) for a in arrays]
    out = BagBatch(batch.n, batch.names, p[:nc], p[nc:2 * nc], *p[2 * nc:])
    for a, b in zip(out.kinds + out.values, p[:2 * nc]):
        assert a.ctypes.data == b.ctypes.data  # (no copy made by the constructor)
    return out, arena


def pinned_narrow(batch: BagBatch):
    """(the narrow form of `batch` whose arrays -- kinds, u32 / u64 values, string bytes, u32 offsets,
    times, maps -- live in pinned memory, the arena that holds them): what a binding's packing arena
    holds for mxp_batch_upload2."""
    from .bags import NarrowBatch
    pb, arena = pinned_batch(batch)
    extra = NarrowBatch(batch)  # (sizes)
    need = (sum(v.nbytes + 64 for v in extra.values32 if v is not None) + extra.str_offsets32.nbytes
            + extra.map_offsets32.nbytes + extra.narrow.nbytes + 4 * 64)
    arena2 = PinnedArena(need)
    nb = NarrowBatch(pb, alloc=arena2.empty)
    return nb, (arena, arena2)


def go_to_upper(s: bytes) -> bytes:
    """strings.ToUpper as the case-insensitive lists apply it (mxp_go_to_upper; stringList.go:59,66,79)."""
    lib = load_library()
    n = ctypes.c_uint64(0)
    cap = 3 * len(s) + 8  # a rune grows to at most 3x its bytes (an invalid byte -> EF BF BD)
    out = ctypes.create_string_buffer(cap)
    rc = lib.mxp_go_to_upper(s, len(s), out, cap, ctypes.byref(n))
    if rc != 0:
        raise MxpError("mxp_go_to_upper failed (%d)" % rc)
    return out.raw[:n.value]


# referenced-attribute conditions (include/mxp.h mxp_attr_ref)
REF_NOKEY, REF_ABSENCE, REF_EXACT, REF_MAP = 0xFFFFFFFF, 1, 2, 16


def fakebag_list(refs_row):
    """FakeBag.ReferencedList form (il/testing/fakebag.go:75-89): sorted "name" / "name[key]"."""
    return sorted({a if k is None else "%s[%s]" % (a, k) for a, k, _ in refs_row})


def protobag_set(refs_row):
    """ProtoBag referencedAttrs form (protoBag.go:149-159): {(name, key or "", condition)}, string maps
    fetched whole not recorded."""
    return {(a, k or "", c) for a, k, c in refs_row if c != REF_MAP}


class MxpError(RuntimeError):
    pass


class Engine:
    """One GPU (or a host-only compiler when device=-1) + one rule set."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _VP()
        rc = self.lib.mxp_engine_create(device, ctypes.byref(h))
        if rc != 0:
            raise MxpError("mxp_engine_create(%d) failed with %d" % (device, rc))
        self.h = h
        self.device = device
        self.rules: List[str] = []
        self.status = np.zeros(0, dtype=np.int32)

    @classmethod
    def member(cls, handle, device: int, rules=()) -> "Engine":
        """A non-owning view of a group member's engine (mxp_group_engine): freed with its group."""
        e = cls.__new__(cls)
        e.lib, e.h, e.device, e._owner = load_library(), _VP(handle), device, False
        e.rules, e.status = list(rules), np.zeros(0, dtype=np.int32)
        return e

    def close(self):
        if self.h and getattr(self, "_owner", True):
            self.lib.mxp_engine_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise MxpError("%s failed (%d): %s" % (what, rc, self.lib.mxp_last_error(self.h).decode(errors="replace")))

    # ------------------------------------------------------------------ configuration
    def set_vocabulary(self, manifest: Dict[str, object]):
        """ChangeVocabulary (evaluator.go:107): manifest name -> ValueType (name or enum value)."""
        names = list(manifest)
        types = [VALUE_TYPES[v] if isinstance(v, str) else int(v) for v in manifest.values()]
        arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        tarr = (ctypes.c_int32 * max(len(types), 1))(*types)
        self._check(self.lib.mxp_vocab_set(self.h, arr, tarr, len(names)), "mxp_vocab_set")
        self.vocab_names = names
        self.rules = []

    def set_vocabulary_finder(self, get_attribute):
        """ChangeVocabulary(finder) (runtime/controller.go:100-102): `get_attribute(name)` is the
        finder's GetAttribute -- a ValueType (name or enum value), or None when the name is not in
        the vocabulary.  The engine asks for each name its rules use, the first time it meets it."""
        def find(_ctx, name):
            v = get_attribute(name.decode())
            return -1 if v is None else (VALUE_TYPES[v] if isinstance(v, str) else int(v))
        self._finder = _FINDER(find)  # (kept alive while the engine may call it)
        self._check(self.lib.mxp_vocab_set_finder(self.h, ctypes.cast(self._finder, _VP), None), "mxp_vocab_set_finder")
        self.vocab_names = None
        self.rules = []

    def vocab_name(self, pos: int) -> str:
        """Name of vocabulary position `pos` (mxp_attr_ref.attr)."""
        return self._text(self.lib.mxp_vocab_name, pos)

    def compile(self, rules: Sequence[str]) -> np.ndarray:
        """Compile + upload a rule set; returns per-rule status (RULE_*)."""
        self.rules = list(rules)
        enc = [r.encode("utf-8", "surrogateescape") for r in self.rules]
        arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        st = np.zeros(len(enc), dtype=np.int32)
        self._check(self.lib.mxp_ruleset_compile(self.h, arr, len(enc), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))),
                    "mxp_ruleset_compile")
        self.status = st
        return st

    def _text(self, fn, rule, cap=1 << 16):
        buf = ctypes.create_string_buffer(cap)
        self._check(fn(self.h, rule, buf, cap), fn.__name__)
        return buf.value.decode("utf-8", "surrogateescape")

    def rule_error(self, rule: int) -> str:
        return self._text(self.lib.mxp_rule_error, rule)

    def rule_il_text(self, rule: int) -> str:
        return self._text(self.lib.mxp_rule_il_text, rule)

    def rule_vm_text(self, rule: int) -> str:
        return self._text(self.lib.mxp_rule_vm_text, rule)

    def rule_types(self, rule: int):
        vt, il = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.mxp_rule_types(self.h, rule, ctypes.byref(vt), ctypes.byref(il)), "mxp_rule_types")
        return vt.value, il.value

    def set_pipeline(self, min_requests: int = 1 << 17, max_chunks: int = 8):
        """Request chunks whose guard-index pass overlaps the next chunk's fill (mxp_set_pipeline)."""
        self._check(self.lib.mxp_set_pipeline(self.h, min_requests, max_chunks), "mxp_set_pipeline")

    def set_timing(self, on: bool = True):
        self._check(self.lib.mxp_set_timing(self.h, int(on)), "mxp_set_timing")

    def kernel_times(self, n_values: int = 2):
        """[guard/VM kernel ms, guard-index kernel ms] of the last device evaluation (timing on); with
        n_values=3 also [2] = 1.0 when it deferred its index pairs (the index kernel and the pair sort
        are then in [0], the fills in [1])."""
        ms = (ctypes.c_float * n_values)()
        n = ctypes.c_uint32()
        self._check(self.lib.mxp_kernel_times(self.h, ms, n_values, ctypes.byref(n)), "mxp_kernel_times")
        return list(ms)[: n.value]

    def wave_times(self, n_waves: int) -> np.ndarray:
        """Profiling hook (MXP_WAVE_TIMES=1 at engine creation): [waves, 8] {start, end, XCC} of the
        last guard-index kernel launch (100 MHz ticks), then 5 phase marks: the end of each of the
        first 4 probe slots and of the queue drain (0 where the wave had fewer slots)."""
        out = np.zeros(8 * n_waves, dtype=np.uint64)
        k = ctypes.c_uint64()
        self._check(self.lib.mxp_debug_wave_times(self.h, out.ctypes.data, out.size, ctypes.byref(k)),
                    "mxp_debug_wave_times")
        return out[:k.value].reshape(-1, 8)

    def bin_stats(self):
        """(bytes of freed batch blocks kept for reuse, the cap) -- mxp_debug_bin."""
        out = (ctypes.c_uint64 * 2)()
        self._check(self.lib.mxp_debug_bin(self.h, out), "mxp_debug_bin")
        return int(out[0]), int(out[1])

    def ruleset_info(self) -> dict:
        """Kernel-side shape of the rule set (guards, continuation templates, column segments)."""
        out = (ctypes.c_uint32 * 10)()
        k = self.lib.mxp_ruleset_info(self.h, out, 10)
        return dict(zip(("guarded", "templated", "templates", "segments", "indexed", "columns", "composite",
                         "aliases", "dense", "value_class_columns"), list(out)[:k]))

    def read_attributes(self) -> list:
        """mxp_ruleset_columns: the attribute names the compiled set reads (the columns to pack),
        plus the resolver's identity attribute and context.protocol once it is configured."""
        n = self.lib.mxp_ruleset_columns(self.h, None, 0)
        arr = (ctypes.c_char_p * max(n, 1))()
        n = self.lib.mxp_ruleset_columns(self.h, arr, n)
        return [arr[i].decode() for i in range(n)]

    # ------------------------------------------------------------------ evaluation
    def eval_batch(self, batch: BagBatch):
        """-> (match, err) uint32 bitmaps, rule-word-major [(R+31)//32, N]."""
        W = (len(self.rules) + 31) // 32
        match = np.zeros((W, batch.n), dtype=np.uint32)
        err = np.zeros((W, batch.n), dtype=np.uint32)
        self._check(self.lib.mxp_eval_batch(self.h, ctypes.byref(batch.c_struct()), match.ctypes.data, err.ctypes.data),
                    "mxp_eval_batch")
        return match, err

    def eval_refs_raw(self, batch: BagBatch, cap: int = 0):
        """mxp_eval_refs without decoding: (ref_off u64[n+1], entries u32[m, 4] = attr, key, cond, 0)."""
        off = np.zeros(batch.n + 1, dtype=np.uint64)
        cap = cap or 16 * max(batch.n, 1)
        while True:
            ents = np.empty((max(cap, 1), 4), dtype=np.uint32)
            rc = self.lib.mxp_eval_refs(self.h, ctypes.byref(batch.c_struct()), None, None, off.ctypes.data,
                                        ents.ctypes.data, cap)
            if rc == 4 and int(off[-1]) > cap:
                cap = int(off[-1])
                continue
            self._check(rc, "mxp_eval_refs")
            return off, ents[:int(off[-1])]

    def eval_refs(self, batch: BagBatch, cap: int = 0):
        """mxp_eval_refs -> (match, err, refs): refs[q] = [(attribute, map key or None, cond)], cond one of
        REF_ABSENCE / REF_EXACT / REF_MAP, sorted by (vocabulary position, key id)."""
        W = (len(self.rules) + 31) // 32
        match = np.zeros((W, batch.n), dtype=np.uint32)
        err = np.zeros((W, batch.n), dtype=np.uint32)
        off = np.zeros(batch.n + 1, dtype=np.uint64)
        cap = cap or 16 * max(batch.n, 1)
        while True:
            ents = np.zeros((max(cap, 1), 4), dtype=np.uint32)
            rc = self.lib.mxp_eval_refs(self.h, ctypes.byref(batch.c_struct()), match.ctypes.data, err.ctypes.data,
                                        off.ctypes.data, ents.ctypes.data, cap)
            if rc == 4 and int(off[-1]) > cap:  # MXP_ERR_NOMEM: retry with the exact size
                cap = int(off[-1])
                continue
            self._check(rc, "mxp_eval_refs")
            break
        return match, err, self._decode_refs(batch.n, off, ents)

    def resolve_refs(self, batch: BagBatch, variety: int, cap: int = 0):
        """mxp_resolve_refs -> (status, err_rule, selected, refs) (see resolve / eval_refs)."""
        n = batch.n
        status = np.zeros(n, dtype=np.uint8)
        err_rule = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n + 1, dtype=np.uint64)
        roff = np.zeros(n + 1, dtype=np.uint64)
        scap, rcap = max(16, n * 4), cap or 16 * max(n, 1)
        while True:
            sel = np.zeros(scap, dtype=np.uint32)
            ents = np.zeros((max(rcap, 1), 4), dtype=np.uint32)
            rc = self.lib.mxp_resolve_refs(self.h, ctypes.byref(batch.c_struct()), variety, status.ctypes.data,
                                           err_rule.ctypes.data, off.ctypes.data, sel.ctypes.data, scap,
                                           roff.ctypes.data, ents.ctypes.data, rcap)
            if rc == 4 and (int(off[n]) > scap or int(roff[n]) > rcap):
                scap, rcap = max(scap, int(off[n])), max(rcap, int(roff[n]))
                continue
            self._check(rc, "mxp_resolve_refs")
            break
        return (status, err_rule, [sel[int(off[q]):int(off[q + 1])] for q in range(n)],
                self._decode_refs(n, roff, ents))

    def _decode_refs(self, n, off, ents):
        keys = {}
        refs = []
        for q in range(n):
            row = []
            for a, k, c, _ in ents[int(off[q]):int(off[q + 1])]:
                key = None
                if k != REF_NOKEY:
                    if k not in keys:
                        keys[k] = self.string_text(int(k))
                    key = keys[k]
                row.append((self.vocab_names[a] if self.vocab_names is not None else self.vocab_name(int(a)), key, int(c)))
            refs.append(row)
        return refs

    def string_text(self, sid: int) -> str:
        buf = ctypes.create_string_buffer(1 << 16)
        self._check(self.lib.mxp_string_text(self.h, sid, buf, 1 << 16), "mxp_string_text")
        return buf.value.decode("utf-8", "surrogateescape")

    def eval_codes(self, batch: BagBatch) -> np.ndarray:
        """Per-pair codes [N, R] (FALSE/TRUE/ERROR/PANIC) via eval_values."""
        _, codes = self.eval_values(batch)
        return codes

    def eval_values(self, batch: BagBatch):
        R = len(self.rules)
        vals = np.zeros((batch.n, R), dtype=np.uint64)
        codes = np.zeros((batch.n, R), dtype=np.uint8)
        self._check(self.lib.mxp_eval_values(self.h, ctypes.byref(batch.c_struct()), vals.ctypes.data, codes.ctypes.data),
                    "mxp_eval_values")
        return vals, codes

    def value_text(self, rule: int, value: int) -> str:
        buf = ctypes.create_string_buffer(1 << 16)
        self._check(self.lib.mxp_value_text(self.h, rule, int(value), buf, 1 << 16), "mxp_value_text")
        return buf.value.decode("utf-8", "surrogateescape")

    def value_kind(self, rule: int, value: int) -> int:
        return self.lib.mxp_value_kind(self.h, rule, int(value))

    def pair_error(self, request: int, rule: int) -> str:
        buf = ctypes.create_string_buffer(1 << 12)
        rc = self.lib.mxp_pair_error(self.h, request, rule, buf, 1 << 12)
        if rc not in (0, 1):
            self._check(rc, "mxp_pair_error")
        return buf.value.decode("utf-8", "surrogateescape")

    # ------------------------------------------------------------------ batched resolver
    RESOLVE_OK, RESOLVE_NO_IDENTITY, RESOLVE_BAD_IDENTITY, RESOLVE_PRED_ERROR = 0, 1, 2, 3

    def set_resolver(self, identity_attr: str, default_ns: str, rule_ns, variety_mask, is_tcp, empty_match):
        """runtime.resolver configuration (mxp_resolver_set): per rule its namespace (rules of a
        namespace contiguous, in resolution order), variety bit mask, TCP flag, empty-match flag."""
        n = len(rule_ns)
        ns = (ctypes.c_char_p * max(n, 1))(*[x.encode() for x in rule_ns])
        vm = np.ascontiguousarray(variety_mask, dtype=np.uint32)
        tcp = np.ascontiguousarray(is_tcp, dtype=np.uint8)
        em = np.ascontiguousarray(empty_match, dtype=np.uint8)
        self._check(self.lib.mxp_resolver_set(self.h, identity_attr.encode(), default_ns.encode(), ns,
                                              vm.ctypes.data, tcp.ctypes.data, em.ctypes.data, n), "mxp_resolver_set")

    def resolve_arrays(self, batch: BagBatch, variety: int, cap: int = 0, ids16: bool = False, pinned: bool = False):
        """mxp_resolve_batch -> (status u8[n], err_rule u32[n], sel_off u64[n + 1], sel_rules u32[...]):
        request q's selected rules are sel_rules[sel_off[q]:sel_off[q + 1]], in resolution order.
        ids16: mxp_resolve_batch_ex with MXP_RESOLVE_IDS_U16 (sel_rules u16).  pinned: the outputs in
        a pinned arena the engine object keeps (DMA straight into them; the arrays are views, valid
        until the next pinned call)."""
        n = batch.n
        cap = cap or max(16, n * 4)
        isz = 2 if ids16 else 4

        def outputs(cap):
            if not pinned:
                return (np.empty(n, dtype=np.uint8), np.empty(n, dtype=np.uint32), np.empty(n + 1, dtype=np.uint64),
                        np.empty(cap, dtype=np.uint16 if ids16 else np.uint32))
            need = n * 13 + 8 + cap * isz + 4 * 64
            if getattr(self, "_out_arena", None) is None or self._out_arena.size < need:
                self._out_arena = PinnedArena(int(need * 1.25))
            a = self._out_arena
            a.used = 0
            return (a.empty(n, np.uint8), a.empty(n, np.uint32), a.empty(n + 1, np.uint64),
                    a.empty(cap, np.uint16 if ids16 else np.uint32))
        for _ in range(2):
            status, err_rule, off, sel = outputs(cap)
            if ids16:
                rc = self.lib.mxp_resolve_batch_ex(self.h, ctypes.byref(batch.c_struct()), variety, 1,
                                                   status.ctypes.data, err_rule.ctypes.data, off.ctypes.data,
                                                   sel.ctypes.data, cap)
            else:
                rc = self.lib.mxp_resolve_batch(self.h, ctypes.byref(batch.c_struct()), variety, status.ctypes.data,
                                                 err_rule.ctypes.data, off.ctypes.data, sel.ctypes.data, cap)
            if rc == 4:  # MXP_ERR_NOMEM: retry with the exact size
                cap = int(off[n])
                continue
            self._check(rc, "mxp_resolve_batch")
            break
        return status, err_rule, off, sel[:int(off[n])]

    def resolve_uploaded(self, db: "DeviceBatch", variety: int, cap: int, ids16: bool = False):
        """mxp_resolve_uploaded: Resolve a batch uploaded before (db is taken over) -> as resolve_arrays."""
        batch, cs = db._src
        n = batch.n
        status, err_rule = np.empty(n, dtype=np.uint8), np.empty(n, dtype=np.uint32)
        off, sel = np.empty(n + 1, dtype=np.uint64), np.empty(max(cap, 1), dtype=np.uint16 if ids16 else np.uint32)
        h, db.h = db.h, None
        self._check(self.lib.mxp_resolve_uploaded(self.h, h, ctypes.byref(cs) if cs is not None else None, variety,
                                                  1 if ids16 else 0,
                                                  status.ctypes.data, err_rule.ctypes.data, off.ctypes.data,
                                                  sel.ctypes.data, cap), "mxp_resolve_uploaded")
        return status, err_rule, off, sel[:int(off[n])]

    def resolve_submit(self, db: "DeviceBatch", variety: int, ids16: bool = False):
        """mxp_resolve_submit: the evaluation of an uploaded batch enqueued (db taken over) -> a job for
        resolve_finish; the engine takes only an upload in between."""
        batch, cs = db._src
        h, db.h = db.h, None
        job = _VP()
        self._check(self.lib.mxp_resolve_submit(self.h, h, ctypes.byref(cs) if cs is not None else None, variety,
                                                1 if ids16 else 0, ctypes.byref(job)), "mxp_resolve_submit")
        return (job, batch.n, ids16)

    def resolve_finish(self, job, cap: int):
        """mxp_resolve_finish -> (status, err_rule, sel_off, sel_rules) as resolve_uploaded."""
        h, n, ids16 = job
        status, err_rule = np.empty(n, dtype=np.uint8), np.empty(n, dtype=np.uint32)
        off, sel = np.empty(n + 1, dtype=np.uint64), np.empty(max(cap, 1), dtype=np.uint16 if ids16 else np.uint32)
        self._check(self.lib.mxp_resolve_finish(h, status.ctypes.data, err_rule.ctypes.data, off.ctypes.data,
                                                sel.ctypes.data, cap), "mxp_resolve_finish")
        return status, err_rule, off, sel[:int(off[n])]

    def resolve(self, batch: BagBatch, variety: int, ids16: bool = False):
        """Resolve every request (mxp_resolve_batch) -> (status u8[n], err_rule u32[n], selected:
        list of per-request rule-id arrays in resolution order)."""
        status, err_rule, off, sel = self.resolve_arrays(batch, variety, ids16=ids16)
        return status, err_rule, [sel[int(off[q]):int(off[q + 1])] for q in range(batch.n)]

    # ------------------------------------------------------------------ list adapter
    def list_create(self, entry_type: int, entries, overrides=()) -> "ListHandle":
        """mxp_list_create: entries / overrides as str or bytes."""
        def arr(xs):
            bs = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x) for x in xs]
            bufs = [ctypes.create_string_buffer(b, len(b) + 1) for b in bs]
            ptrs = (ctypes.c_char_p * max(len(bs), 1))(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs])
            lens = np.array([len(b) for b in bs] or [0], dtype=np.uint32)
            return bufs, ptrs, lens, len(bs)
        eb, ep, el, en = arr(entries)
        ob, op, ol, on = arr(overrides)
        h = _VP()
        self._check(self.lib.mxp_list_create(self.h, entry_type, ep, el.ctypes.data, en, op, ol.ctypes.data, on,
                                             ctypes.byref(h)), "mxp_list_create")
        return ListHandle(self, h)

    # ------------------------------------------------------------------ memquota
    def quota_create(self, max_amount, valid_duration_ns) -> "QuotaHandle":
        mx = np.ascontiguousarray(max_amount, dtype=np.int64)
        vd = np.ascontiguousarray(valid_duration_ns, dtype=np.int64)
        h = _VP()
        self._check(self.lib.mxp_quota_create(self.h, len(mx), mx.ctypes.data, vd.ctypes.data, ctypes.byref(h)),
                    "mxp_quota_create")
        return QuotaHandle(self, h)

    def error_count(self) -> int:
        return int(self.lib.mxp_error_count(self.h))

    # ------------------------------------------------------------------ device-resident batches
    def pack_host(self, batch: BagBatch) -> dict:
        """Host half of upload alone (mxp_batch_pack_host): packed bytes, overlay strings / byte strings."""
        out = (ctypes.c_uint64 * 3)()
        self._check(self.lib.mxp_batch_pack_host(self.h, ctypes.byref(batch.c_struct()), out, 3), "mxp_batch_pack_host")
        return {"bytes": out[0], "overlay_strings": out[1], "overlay_bytes": out[2]}

    def upload(self, batch: BagBatch, no_wait: bool = False) -> "DeviceBatch":
        """mxp_batch_upload; no_wait: mxp_batch_upload_ex(MXP_UPLOAD_NO_WAIT) -- the batch's arrays
        stay unchanged until DeviceBatch.wait_copied() (the c_struct keeps them referenced)."""
        h = _VP()
        cs = batch.c_struct()
        if no_wait:
            rc = self.lib.mxp_batch_upload_ex(self.h, ctypes.byref(cs), 1, ctypes.byref(h))
        else:
            rc = self.lib.mxp_batch_upload(self.h, ctypes.byref(cs), ctypes.byref(h))
        self._check(rc, "mxp_batch_upload")
        db = DeviceBatch(self, h, batch.n)
        db._src = (batch, cs)  # (the host arrays the copies read)
        return db


def _upload2(self, nb, no_wait: bool = False) -> "DeviceBatch":
    """mxp_batch_upload2: a NarrowBatch (bags.py) uploaded narrow and widened on the device."""
    h = _VP()
    cs = nb.c_struct()
    self._check(self.lib.mxp_batch_upload2(self.h, ctypes.byref(cs), 1 if no_wait else 0, ctypes.byref(h)),
                "mxp_batch_upload2")
    db = DeviceBatch(self, h, nb.n)
    db._src = (nb, None)  # (resolve_uploaded passes NULL: the engine keeps the host view)
    return db


Engine.upload2 = _upload2


class DeviceBatch:
    def __init__(self, engine: Engine, h, n: int):
        self.engine = engine
        self.h = h
        self.n = n

    def wait_copied(self):
        """mxp_batch_wait_copied: the batch's host arrays are free again (after a no_wait upload).
        (DeviceBatch)"""
        self.engine._check(self.engine.lib.mxp_batch_wait_copied(self.h), "mxp_batch_wait_copied")

    def eval(self, d_match: int, d_err: int, stream: int = 0):
        """Enqueue one evaluation writing device bitmaps (raw device pointers as ints)."""
        e = self.engine
        e._check(e.lib.mxp_batch_eval_device(e.h, self.h, _VP(stream or None), _VP(d_match), _VP(d_err)),
                 "mxp_batch_eval_device")

    def eval_hits(self, d_match: int, d_err: int, d_hits: int, stream: int = 0):
        """eval() plus fused per-rule hit counters: d_hits[rule] += true pairs (device u64)."""
        e = self.engine
        e._check(e.lib.mxp_batch_eval_device_hits(e.h, self.h, _VP(stream or None), _VP(d_match), _VP(d_err),
                                                  _VP(d_hits)), "mxp_batch_eval_device_hits")

    def eval_compact(self, d_match: int, d_req_err: int, d_hits: int = 0, stream: int = 0):
        """eval_hits() with compact error output: no error bitmap, d_req_err[q] (device u8) = 1 when some
        rule fails for request q; d_hits 0 = no counters."""
        e = self.engine
        e._check(e.lib.mxp_batch_eval_device_compact(e.h, self.h, _VP(stream or None), _VP(d_match), _VP(d_req_err),
                                                     _VP(d_hits or None)), "mxp_batch_eval_device_compact")

    def free(self):
        if self.h:
            self.engine.lib.mxp_batch_free(self.engine.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def bits_to_codes(match: np.ndarray, err: np.ndarray, n_rules: int) -> np.ndarray:
    """Unpack rule-word-major bitmaps into [N, R] codes (error and panic both -> ERROR)."""
    W, n = match.shape
    shifts = np.arange(32, dtype=np.uint32)
    m = ((match.T[:, :, None] >> shifts) & 1).reshape(n, W * 32)[:, :n_rules]
    e = ((err.T[:, :, None] >> shifts) & 1).reshape(n, W * 32)[:, :n_rules]
    return np.where(e != 0, ERROR, m).astype(np.uint8)


class TypeChecker:
    """expr.TypeChecker (mixer/pkg/expr/evaluator.go:33-42) as evaluator.checker implements it
    (mixer/pkg/il/evaluator/checker.go:29-46): the engine's own front end and type check
    (mxp_ruleset_compile on a host-only engine, mxp_rule_types), no device needed.  `finder` maps
    attribute names to ValueTypes (names or enum values), like an AttributeDescriptorFinder."""

    _NAMES = {v: k for k, v in VALUE_TYPES.items()}

    def __init__(self):
        self.eng = Engine(-1)

    def eval_type(self, expression: str, finder: Dict[str, object]):
        """-> (ValueType name, error text or None): EvalType (checker.go:29-35)."""
        self.eng.set_vocabulary(finder)
        st = int(self.eng.compile([expression])[0])
        if st == RULE_PARSE_ERROR:
            return "VALUE_TYPE_UNSPECIFIED", "failed to parse expression '%s': %s" % (expression, self.eng.rule_error(0))
        if st in (RULE_TYPE_ERROR, RULE_COMPILE_PANIC):
            return "VALUE_TYPE_UNSPECIFIED", self.eng.rule_error(0)
        return self._NAMES[self.eng.rule_types(0)[0]], None

    def assert_type(self, expression: str, finder: Dict[str, object], expected: str):
        """-> error text or None: AssertType (checker.go:37-44)."""
        t, err = self.eval_type(expression, finder)
        if err is not None:
            return err
        if t != expected:
            return "expression '%s' evaluated to type %s, expected type %s" % (expression, t, expected)
        return None


class Evaluator:
    """expr.Evaluator (mixer/pkg/expr/evaluator.go:25-31) for single bags, on the GPU engine.

    Every distinct expression is compiled once (like evaluator.IL's cache, but unbounded) into a
    one-rule engine; each call evaluates one bag."""

    def __init__(self, manifest: Dict[str, object], device: int = 0):
        self.manifest = dict(manifest)
        self.device = device
        self._engines: Dict[str, Engine] = {}

    def change_vocabulary(self, manifest: Dict[str, object]):
        self.manifest = dict(manifest)
        self._engines.clear()

    def _engine(self, text: str) -> Engine:
        e = self._engines.get(text)
        if e is None:
            e = Engine(self.device)
            e.set_vocabulary(self.manifest)
            e.compile([text])
            self._engines[text] = e
        return e

    def eval(self, text: str, bag: dict):
        """-> ('ok', python value) | ('error', msg) | ('panic', msg)."""
        e = self._engine(text)
        st = int(e.status[0])
        if st not in (RULE_OK,):
            return ("panic" if st == RULE_COMPILE_PANIC else "error"), e.rule_error(0)
        b = BagBatch.from_bags([bag])
        vals, codes = e.eval_values(b)
        c = int(codes[0, 0])
        if c in (ERROR, PANIC):
            msg = e.pair_error(0, 0)
            if c == PANIC and msg == "interpreter.Result: result is not bool":
                c = FALSE  # Eval (not EvalPredicate): a non-bool result is a value
            else:
                return ("panic" if c == PANIC else "error"), msg
        return "ok", decode_value(e, 0, int(vals[0, 0]))

    def eval_predicate(self, text: str, bag: dict):
        e = self._engine(text)
        st = int(e.status[0])
        if st != RULE_OK:
            return ("panic" if st == RULE_COMPILE_PANIC else "error"), e.rule_error(0)
        b = BagBatch.from_bags([bag])
        match, err = e.eval_batch(b)
        if err[0, 0] & 1:
            msg = e.pair_error(0, 0)
            return ("panic" if msg in PANIC_TEXTS else "error"), msg
        return "ok", bool(match[0, 0] & 1)


PANIC_TEXTS = {"Unknown map type", "reflect: Call using a value of the wrong type",
               "interpreter.Result: result is not bool", "interface conversion: interface {} is not string",
               "runtime error: index out of range"}


class _Value(ctypes.Structure):  # mxp_value (mxp.h)
    _fields_ = [("kind", ctypes.c_uint32), ("n", ctypes.c_uint32), ("i", ctypes.c_int64), ("d", ctypes.c_double),
                ("nsec", ctypes.c_int32), ("pad", ctypes.c_uint32)]


def decode_value(e: Engine, rule: int, v: int):
    """Engine result register -> Python Go-model value (interpreter.Result.AsInterface), through
    mxp_value_decode: bool, GoInt64, GoDuration, GoFloat64, str, bytes, GoTime, dict."""
    from .bags import GoDuration, GoFloat64, GoInt64, GoTime
    out = _Value()
    cap = 1 << 12
    while True:
        buf = ctypes.create_string_buffer(cap)
        rc = e.lib.mxp_value_decode(e.h, rule, v, ctypes.addressof(out), buf, cap)
        if rc != 4:  # MXP_ERR_NOMEM: again with room for out.n bytes
            break
        cap = out.n + 16
    e._check(rc, "mxp_value_decode")
    raw = buf.raw[:out.n]
    k = out.kind
    if k == 4:  # MXP_BOOL
        return bool(out.i)
    if k == 2:
        return GoInt64(out.i)
    if k == 3:
        return GoFloat64(out.d)
    if k == 5:
        return GoDuration(out.i)
    if k == 1:
        return raw.decode("utf-8", "surrogateescape")
    if k == 7:
        return raw
    if k == 6:
        return GoTime(out.i, out.nsec)
    if k == 8:  # string map: (u32 len, bytes) key / value runs
        m, at = {}, 0
        for _ in range(out.i):
            kv = []
            for _ in range(2):
                n = int.from_bytes(raw[at:at + 4], "little")
                kv.append(raw[at + 4:at + 4 + n].decode("utf-8", "surrogateescape"))
                at += 4 + n
            m[kv[0]] = kv[1]
        return m
    raise MxpError("value of kind %d" % k)


class ListHandle:
    """A compiled list (mxp_list): HandleListEntry for batches of symbols."""
    STRINGS, CASE_INSENSITIVE_STRINGS, IP_ADDRESSES, REGEX = 0, 1, 2, 3

    def __init__(self, eng: Engine, h):
        self.eng, self.h = eng, h

    def num_entries(self) -> int:
        return int(self.eng.lib.mxp_list_entries(self.h))

    def regex_dispatch(self):
        """(patterns dispatched by their literal prefix, distinct prefixes) of a REGEX list."""
        out = (ctypes.c_uint32 * 2)()
        self.eng.lib.mxp_list_regex_dispatch(self.h, out)
        return int(out[0]), int(out[1])

    def regex_parts(self):
        """(automata, of which bit-parallel NFAs) of a REGEX list."""
        out = (ctypes.c_uint32 * 2)()
        self.eng.lib.mxp_list_regex_parts(self.h, out)
        return int(out[0]), int(out[1])

    def check(self, symbols, blacklist: bool = False) -> np.ndarray:
        """google.rpc codes (0 OK, 3 INVALID_ARGUMENT, 5 NOT_FOUND, 7 PERMISSION_DENIED) per symbol."""
        bs = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x) for x in symbols]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
        blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
        codes = np.zeros(len(bs), dtype=np.int32)
        self.eng._check(self.eng.lib.mxp_list_check(self.eng.h, self.h, int(blacklist), blob.ctypes.data,
                                                    off.ctypes.data, len(bs), codes.ctypes.data), "mxp_list_check")
        return codes

    def check_entries(self, engine: "Engine", batch, value_rule: int, blacklist: bool = False, texts: bool = False):
        """mxp_listentry_check: the listentry instance's Value = Eval(rule value_rule of `engine`) per
        request, checked against this list in one device pass; -1 where Eval failed.  texts: also
        each request's Value text (mxp_value_text of the returned registers; None where Eval failed),
        the symbol HandleListEntry's messages print."""
        codes = np.zeros(batch.n, dtype=np.int32)
        vals = np.zeros(batch.n if texts else 0, dtype=np.uint64)
        engine._check(engine.lib.mxp_listentry_check(engine.h, self.h, int(blacklist), ctypes.byref(batch.c_struct()),
                                                      value_rule, codes.ctypes.data, vals.ctypes.data if texts else None),
                      "mxp_listentry_check")
        if not texts:
            return codes
        return codes, [engine.value_text(value_rule, int(v)) if c >= 0 else None for c, v in zip(codes, vals)]

    def check_device(self, d_sym: int, d_off: int, n: int, stream: int, d_codes: int, blacklist: bool = False):
        """mxp_list_check_device: symbols (blob with >= 16 bytes of slack) and codes in device memory."""
        self.eng._check(self.eng.lib.mxp_list_check_device(self.eng.h, self.h, int(blacklist), d_sym, d_off, n,
                                                           stream, d_codes), "mxp_list_check_device")

    def __del__(self):
        try:
            if self.h and not getattr(self, "_view", False):
                self.eng.lib.mxp_list_destroy(self.eng.h, self.h)
                self.h = None
        except Exception:
            pass


def regex_match_host(pattern, subject):
    """mxp_regex_match_host -> (status, text): 1 / 0 match, -1 syntax error (Go text), -2 unsupported,
    -3 DFA too big."""
    lib = load_library()
    p = pattern.encode("utf-8", "surrogateescape") if isinstance(pattern, str) else bytes(pattern)
    s = subject.encode("utf-8", "surrogateescape") if isinstance(subject, str) else bytes(subject)
    buf = ctypes.create_string_buffer(1024)
    rc = lib.mxp_regex_match_host(p, len(p), s, len(s), buf, 1024)
    return rc, buf.value.decode("utf-8", "surrogateescape")


class QuotaHandle:
    """Batched memquota state (mxp_quota): HandleQuota for requests in arrival order."""

    def __init__(self, eng: Engine, h):
        self.eng, self.h = eng, h

    def alloc(self, keys, amounts, best_effort, now_ns: int) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        a = np.ascontiguousarray(amounts, dtype=np.int64)
        b = np.ascontiguousarray(best_effort, dtype=np.uint8)
        out = np.zeros(len(k), dtype=np.int64)
        self.eng._check(self.eng.lib.mxp_quota_alloc(self.eng.h, self.h, len(k), k.ctypes.data, a.ctypes.data,
                                                     b.ctypes.data, int(now_ns), out.ctypes.data), "mxp_quota_alloc")
        return out

    def alloc_device(self, n, d_keys, d_amounts, d_be, now_ns, stream, d_granted, d_delta=None):
        self.eng._check(self.eng.lib.mxp_quota_alloc_device(self.eng.h, self.h, n, d_keys, d_amounts, d_be,
                                                            int(now_ns), stream, d_granted, d_delta or None),
                        "mxp_quota_alloc_device")

    def __del__(self):
        try:
            if self.h:
                self.eng.lib.mxp_quota_destroy(self.eng.h, self.h)
                self.h = None
        except Exception:
            pass


REDUCE_NONE, REDUCE_RCCL, REDUCE_HOST = 0, 1, 2
GROUP_HOST_REDUCE, GROUP_RCCL_SINGLE = 1, 2


def shard_bounds(n_total: int, member: int, n_members: int):
    """mxp_group_shard_bounds: member's contiguous [lo, hi) of n_total requests."""
    lib = load_library()
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    lib.mxp_group_shard_bounds(n_total, member, n_members, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def key_owners(weights, n_members: int) -> np.ndarray:
    """mxp_group_key_owners: each memquota key's owner member, longest-processing-time first."""
    lib = load_library()
    w = np.ascontiguousarray(weights, dtype=np.float64)
    out = np.zeros(len(w), dtype=np.uint32)
    rc = lib.mxp_group_key_owners(w.ctypes.data, len(w), n_members, out.ctypes.data)
    if rc != 0:
        raise MxpError("mxp_group_key_owners failed (%d)" % rc)
    return out


class Group:
    """A device group (include/mxp_group.h): one engine per device, request shards evaluated on all
    members at once, the step's counters (hits[R] ++ quota_delta[K]) summed by one all-reduce
    (RCCL, or the host when RCCL is unavailable or a device repeats)."""

    def __init__(self, devices: Sequence[int], flags: int = 0):
        self.lib = load_library()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = _VP()
        rc = self.lib.mxp_group_create(devs, len(devices), flags, ctypes.byref(h))
        if rc != 0:
            raise MxpError("mxp_group_create(%s) failed (%d): %s" % (list(devices), rc,
                                                                   self.lib.mxp_group_last_error(None).decode()))
        self.h, self.devices = h, list(devices)
        self.n = len(devices)
        self.rules: List[str] = []
        self.note = self.lib.mxp_group_last_error(h).decode()  # (why the reduction is on the host, if it is)

    def close(self):
        if self.h:
            self.lib.mxp_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise MxpError("%s failed (%d): %s" % (what, rc, self.lib.mxp_group_last_error(self.h).decode(errors="replace")))

    @property
    def reduce_mode(self) -> int:
        return int(self.lib.mxp_group_reduce_mode(self.h))

    def engine(self, k: int) -> Engine:
        """Member k's engine (a view: per-pair error texts, rule texts, values, timing)."""
        return Engine.member(self.lib.mxp_group_engine(self.h, k), self.devices[k], self.rules)

    def stream(self, k: int) -> int:
        return int(self.lib.mxp_group_stream(self.h, k) or 0)

    def locate(self, request: int):
        k, q = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.mxp_group_locate(self.h, request, ctypes.byref(k), ctypes.byref(q)), "mxp_group_locate")
        return k.value, q.value

    # ------------------------------------------------------------------ configuration
    def set_vocabulary(self, manifest: Dict[str, object]):
        names = list(manifest)
        types = [VALUE_TYPES[v] if isinstance(v, str) else int(v) for v in manifest.values()]
        arr = (ctypes.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        tarr = (ctypes.c_int32 * max(len(types), 1))(*types)
        self._check(self.lib.mxp_group_vocab_set(self.h, arr, tarr, len(names)), "mxp_group_vocab_set")

    def set_vocabulary_finder(self, get_attribute):
        def find(_ctx, name):
            v = get_attribute(name.decode())
            return -1 if v is None else (VALUE_TYPES[v] if isinstance(v, str) else int(v))
        self._finder = _FINDER(find)
        self._check(self.lib.mxp_group_vocab_set_finder(self.h, ctypes.cast(self._finder, _VP), None),
                    "mxp_group_vocab_set_finder")

    def compile(self, rules: Sequence[str]) -> np.ndarray:
        self.rules = list(rules)
        enc = [r.encode("utf-8", "surrogateescape") for r in self.rules]
        arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        st = np.zeros(len(enc), dtype=np.int32)
        self._check(self.lib.mxp_group_ruleset_compile(self.h, arr, len(enc), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))),
                    "mxp_group_ruleset_compile")
        return st

    def set_resolver(self, identity_attr: str, default_ns: str, rule_ns, variety_mask, is_tcp, empty_match):
        n = len(rule_ns)
        ns = (ctypes.c_char_p * max(n, 1))(*[x.encode() for x in rule_ns])
        vm = np.ascontiguousarray(variety_mask, dtype=np.uint32)
        tcp = np.ascontiguousarray(is_tcp, dtype=np.uint8)
        em = np.ascontiguousarray(empty_match, dtype=np.uint8)
        self._check(self.lib.mxp_group_resolver_set(self.h, identity_attr.encode(), default_ns.encode(), ns,
                                                    vm.ctypes.data, tcp.ctypes.data, em.ctypes.data, n),
                    "mxp_group_resolver_set")

    # ------------------------------------------------------------------ device-resident shards
    def _shards(self, shards):
        cs = [b.c_struct() for b in shards]
        arr = (_VP * len(cs))(*[ctypes.addressof(c) for c in cs])
        return cs, arr

    def upload(self, shards: Sequence[BagBatch], no_wait: bool = False) -> "GroupBatch":
        """mxp_group_upload: shards[k] -> member k."""
        cs, arr = self._shards(shards)
        h = _VP()
        self._check(self.lib.mxp_group_upload(self.h, arr, len(cs), 1 if no_wait else 0, ctypes.byref(h)),
                    "mxp_group_upload")
        gb = GroupBatch(self, h, [b.n for b in shards])
        gb._src = (list(shards), cs)
        return gb

    def upload2(self, shards, no_wait: bool = False) -> "GroupBatch":
        """mxp_group_upload2: NarrowBatch shards (bags.py), member k's = shards[k]."""
        cs = [b.c_struct() for b in shards]
        arr = (_VP * len(cs))(*[ctypes.addressof(c) for c in cs])
        h = _VP()
        self._check(self.lib.mxp_group_upload2(self.h, arr, len(cs), 1 if no_wait else 0, ctypes.byref(h)),
                    "mxp_group_upload2")
        gb = GroupBatch(self, h, [b.n for b in shards])
        gb._src = (list(shards), None)  # (mxp_group_resolve_uploaded: shards NULL, the members' host views)
        return gb

    def upload_split(self, batch: BagBatch) -> "GroupBatch":
        cs = batch.c_struct()
        h = _VP()
        self._check(self.lib.mxp_group_upload_split(self.h, ctypes.byref(cs), 0, ctypes.byref(h)), "mxp_group_upload_split")
        return GroupBatch(self, h, [self.lib.mxp_group_batch_requests(h, k) for k in range(self.n)])

    def eval(self, gb: "GroupBatch", err_bitmap: bool = False):
        self._check(self.lib.mxp_group_eval(self.h, gb.h, 1 if err_bitmap else 0), "mxp_group_eval")

    def download(self, k: int, n: int, err_bitmap: bool = False):
        """Member k's last results: (match [W, n] u32, err [W, n] u32 or req_err [n] u8)."""
        W = (len(self.rules) + 31) // 32
        match = np.zeros((W, n), dtype=np.uint32)
        if err_bitmap:
            err = np.zeros((W, n), dtype=np.uint32)
            self._check(self.lib.mxp_group_download(self.h, k, match.ctypes.data, err.ctypes.data, None), "mxp_group_download")
        else:
            err = np.zeros(n, dtype=np.uint8)
            self._check(self.lib.mxp_group_download(self.h, k, match.ctypes.data, None, err.ctypes.data), "mxp_group_download")
        return match, err

    # ------------------------------------------------------------------ counters
    def reduce(self):
        self._check(self.lib.mxp_group_reduce(self.h), "mxp_group_reduce")

    def counters(self, n_keys: int = 0):
        hits = np.zeros(len(self.rules), dtype=np.uint64)
        delta = np.zeros(n_keys, dtype=np.int64)
        self._check(self.lib.mxp_group_counters(self.h, hits.ctypes.data, delta.ctypes.data if n_keys else None),
                    "mxp_group_counters")
        return hits, delta

    def counters_reset(self):
        self._check(self.lib.mxp_group_counters_reset(self.h), "mxp_group_counters_reset")

    def sync(self):
        self._check(self.lib.mxp_group_sync(self.h), "mxp_group_sync")

    # ------------------------------------------------------------------ memquota
    def quota_create(self, max_amount, valid_duration_ns, owner=None) -> "GroupQuota":
        mx = np.ascontiguousarray(max_amount, dtype=np.int64)
        vd = np.ascontiguousarray(valid_duration_ns, dtype=np.int64)
        own = None if owner is None else np.ascontiguousarray(owner, dtype=np.uint32)
        h = _VP()
        self._check(self.lib.mxp_group_quota_create(self.h, len(mx), mx.ctypes.data, vd.ctypes.data,
                                                    own.ctypes.data if own is not None else None, ctypes.byref(h)),
                    "mxp_group_quota_create")
        return GroupQuota(self, h, len(mx))

    # ------------------------------------------------------------------ Resolve
    def resolve_arrays(self, shards: Sequence[BagBatch], variety: int, cap: int = 0, ids16: bool = False, out=None,
                       uploaded: "GroupBatch" = None):
        """mxp_group_resolve_batch over shards (member k's requests = shards[k]) -> (status, err_rule,
        sel_off, sel_rules) of the concatenated batch.  out: preallocated (status, err_rule, sel_off,
        sel) arrays (e.g. pinned), reused when large enough.  uploaded: the shards' GroupBatch from an
        earlier upload (mxp_group_resolve_uploaded; taken over -- no retry when cap is short)."""
        n = sum(b.n for b in shards) if shards is not None else uploaded.n
        if uploaded is None:
            cs, arr = self._shards(shards)
        elif uploaded._src[1] is None:  # (narrow uploads: the members keep the host views)
            cs, arr = [None] * self.n, None
        else:  # (the very structs the shards were uploaded from)
            cs = uploaded._src[1]
            arr = (_VP * len(cs))(*[ctypes.addressof(c) for c in cs])
        cap = cap or max(16, n * 4)
        for _ in range(2):
            if out is not None and len(out[3]) >= cap:
                status, err_rule, off, sel = out
            else:
                status, err_rule, off = (np.empty(n, dtype=np.uint8), np.empty(n, dtype=np.uint32),
                                         np.empty(n + 1, dtype=np.uint64))
                sel = np.empty(cap, dtype=np.uint16 if ids16 else np.uint32)
            if uploaded is not None:
                h, uploaded.h = uploaded.h, None
                rc = self.lib.mxp_group_resolve_uploaded(self.h, h, arr, len(cs), variety, 1 if ids16 else 0,
                                                         status.ctypes.data, err_rule.ctypes.data, off.ctypes.data,
                                                         sel.ctypes.data, len(sel))
                self._check(rc, "mxp_group_resolve_uploaded")
                break
            rc = self.lib.mxp_group_resolve_batch(self.h, arr, len(cs), variety, 1 if ids16 else 0, status.ctypes.data,
                                                  err_rule.ctypes.data, off.ctypes.data, sel.ctypes.data, len(sel))
            if rc == 4:
                cap = int(off[n])
                out = None
                continue
            self._check(rc, "mxp_group_resolve_batch")
            break
        return status[:n], err_rule[:n], off[:n + 1], sel[:int(off[n])]

    def resolve_submit(self, uploaded: "GroupBatch", variety: int, ids16: bool = False):
        """mxp_group_resolve_submit: every member's evaluation of the uploaded shards enqueued (taken
        over) -> a job for resolve_finish; only an upload may come in between."""
        if uploaded._src[1] is None:  # (narrow uploads: the members keep the host views)
            arr = None
        else:
            cs = uploaded._src[1]
            arr = (_VP * len(cs))(*[ctypes.addressof(c) for c in cs])
        h, uploaded.h = uploaded.h, None
        job = _VP()
        self._check(self.lib.mxp_group_resolve_submit(self.h, h, arr, self.n, variety, 1 if ids16 else 0,
                                                      ctypes.byref(job)), "mxp_group_resolve_submit")
        return (job, uploaded.n, ids16, uploaded._src)

    def resolve_finish(self, job, cap: int, out=None):
        """mxp_group_resolve_finish -> (status, err_rule, sel_off, sel_rules) of the whole batch."""
        h, n, ids16, _src = job
        if out is not None and len(out[3]) >= cap:
            status, err_rule, off, sel = out
        else:
            status, err_rule, off = (np.empty(n, dtype=np.uint8), np.empty(n, dtype=np.uint32),
                                     np.empty(n + 1, dtype=np.uint64))
            sel = np.empty(max(cap, 1), dtype=np.uint16 if ids16 else np.uint32)
        self._check(self.lib.mxp_group_resolve_finish(self.h, h, status.ctypes.data, err_rule.ctypes.data,
                                                      off.ctypes.data, sel.ctypes.data, len(sel)),
                    "mxp_group_resolve_finish")
        return status[:n], err_rule[:n], off[:n + 1], sel[:int(off[n])]

    def resolve(self, shards: Sequence[BagBatch], variety: int, ids16: bool = False):
        status, err_rule, off, sel = self.resolve_arrays(shards, variety, ids16=ids16)
        return status, err_rule, [sel[int(off[q]):int(off[q + 1])] for q in range(len(status))]

    def pair_error(self, request: int, rule: int) -> str:
        buf = ctypes.create_string_buffer(1 << 12)
        rc = self.lib.mxp_group_pair_error(self.h, request, rule, buf, 1 << 12)
        if rc not in (0, 1):
            self._check(rc, "mxp_group_pair_error")
        return buf.value.decode("utf-8", "surrogateescape")

    # ------------------------------------------------------------------ lists
    def list_create(self, entry_type: int, entries, overrides=()) -> "GroupList":
        def arr(xs):
            bs = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x) for x in xs]
            bufs = [ctypes.create_string_buffer(b, len(b) + 1) for b in bs]
            ptrs = (ctypes.c_char_p * max(len(bs), 1))(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs])
            lens = np.array([len(b) for b in bs] or [0], dtype=np.uint32)
            return bufs, ptrs, lens, len(bs)
        eb, ep, el, en = arr(entries)
        ob, op, ol, on = arr(overrides)
        h = _VP()
        self._check(self.lib.mxp_group_list_create(self.h, entry_type, ep, el.ctypes.data, en, op, ol.ctypes.data, on,
                                                   ctypes.byref(h)), "mxp_group_list_create")
        return GroupList(self, h)


class GroupBatch:
    def __init__(self, group: Group, h, counts):
        self.group, self.h, self.counts = group, h, list(counts)

    @property
    def n(self) -> int:
        return sum(self.counts)

    def wait_copied(self):
        self.group._check(self.group.lib.mxp_group_batch_wait_copied(self.h), "mxp_group_batch_wait_copied")

    def free(self):
        if self.h:
            self.group.lib.mxp_group_batch_free(self.group.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class GroupQuota:
    """memquota keys replicated on every member, each key's requests replayed by its owner."""

    def __init__(self, group: Group, h, n_keys: int):
        self.group, self.h, self.n_keys = group, h, n_keys

    def upload(self, keys, amounts, best_effort) -> "GroupQuotaBatch":
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        a = np.ascontiguousarray(amounts, dtype=np.int64)
        b = np.ascontiguousarray(best_effort, dtype=np.uint8)
        h = _VP()
        g = self.group
        g._check(g.lib.mxp_group_quota_upload(g.h, self.h, len(k), k.ctypes.data, a.ctypes.data, b.ctypes.data,
                                              ctypes.byref(h)), "mxp_group_quota_upload")
        return GroupQuotaBatch(self, h, len(k))

    def eval(self, qb: "GroupQuotaBatch", now_ns: int):
        g = self.group
        g._check(g.lib.mxp_group_quota_eval(g.h, self.h, qb.h, int(now_ns)), "mxp_group_quota_eval")

    def alloc(self, keys, amounts, best_effort, now_ns: int) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        a = np.ascontiguousarray(amounts, dtype=np.int64)
        b = np.ascontiguousarray(best_effort, dtype=np.uint8)
        out = np.zeros(len(k), dtype=np.int64)
        g = self.group
        g._check(g.lib.mxp_group_quota_alloc(g.h, self.h, len(k), k.ctypes.data, a.ctypes.data, b.ctypes.data,
                                             int(now_ns), out.ctypes.data), "mxp_group_quota_alloc")
        return out

    def __del__(self):
        try:
            if self.h:
                self.group.lib.mxp_group_quota_destroy(self.group.h, self.h)
                self.h = None
        except Exception:
            pass


class GroupQuotaBatch:
    def __init__(self, quota: GroupQuota, h, n: int):
        self.quota, self.h, self.n = quota, h, n

    def requests(self, k: int) -> int:
        return int(self.quota.group.lib.mxp_group_quota_batch_requests(self.h, k))

    def granted(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.int64)
        g = self.quota.group
        g._check(g.lib.mxp_group_quota_granted(g.h, self.h, out.ctypes.data), "mxp_group_quota_granted")
        return out

    def free(self):
        if self.h:
            self.quota.group.lib.mxp_group_quota_batch_free(self.quota.group.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class GroupList:
    def __init__(self, group: Group, h):
        self.group, self.h = group, h

    def member(self, k: int) -> ListHandle:
        """Member k's list (non-owning view), for check_device on that member's engine."""
        lh = ListHandle.__new__(ListHandle)
        lh.eng, lh.h, lh._view = self.group.engine(k), _VP(self.group.lib.mxp_group_list_member(self.h, k)), True
        return lh

    def check(self, symbols, blacklist: bool = False) -> np.ndarray:
        bs = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else bytes(x) for x in symbols]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
        blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
        codes = np.zeros(len(bs), dtype=np.int32)
        g = self.group
        g._check(g.lib.mxp_group_list_check(g.h, self.h, int(blacklist), blob.ctypes.data, off.ctypes.data, len(bs),
                                            codes.ctypes.data), "mxp_group_list_check")
        return codes

    def check_device(self, d_syms, d_offs, ns, d_codes, blacklist: bool = False):
        """mxp_group_list_check_device: per member k, n[k] device-resident symbols (raw pointers) ->
        device codes, enqueued on the members' streams."""
        G = self.group.n
        arr = lambda xs: (_VP * G)(*[_VP(int(x)) for x in xs])
        n = (ctypes.c_uint32 * G)(*[int(x) for x in ns])
        g = self.group
        g._check(g.lib.mxp_group_list_check_device(g.h, self.h, int(blacklist), arr(d_syms), arr(d_offs), n,
                                                   arr(d_codes)), "mxp_group_list_check_device")

    def __del__(self):
        try:
            if self.h:
                self.group.lib.mxp_group_list_destroy(self.group.h, self.h)
                self.h = None
        except Exception:
            pass
