"""Wire form of request attributes: `CompressedAttributes` messages (istio.io/api mixer/v1
attributes.proto) flattened into the CSR arrays of include/mxp_batch.h `mxp_wire_batch`, and their
decoding by the engine (mxp_wire_decode) into a columnar BagBatch.

A message is a dict with the proto's fields, keyed by dictionary index (>= 0: global word list,
< 0: the message's own `words`, slot -index-1):

    {"words": [...], "strings": {k: v}, "int64s": {k: i}, "doubles": {k: f}, "bools": {k: b},
     "timestamps": {k: (sec, nsec)}, "durations": {k: ns}, "bytes": {k: b"..."},
     "string_maps": {k: {kk: vv}}}
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import numpy as np

from .bags import BagBatch, _CBatch

_P = ctypes.c_void_p


class _CWire(ctypes.Structure):
    _fields_ = [("n_requests", ctypes.c_uint32), ("n_global", ctypes.c_uint32),
                ("global_bytes", _P), ("global_offsets", _P),
                ("words_off", _P), ("word_bytes", _P), ("word_offsets", _P),
                ("str_off", _P), ("str_key", _P), ("str_val", _P),
                ("i64_off", _P), ("i64_key", _P), ("i64_val", _P),
                ("dbl_off", _P), ("dbl_key", _P), ("dbl_val", _P),
                ("bool_off", _P), ("bool_key", _P), ("bool_val", _P),
                ("ts_off", _P), ("ts_key", _P), ("ts_sec", _P), ("ts_nsec", _P),
                ("dur_off", _P), ("dur_key", _P), ("dur_val", _P),
                ("byt_off", _P), ("byt_key", _P), ("byt_val_off", _P), ("byt_bytes", _P),
                ("sm_off", _P), ("sm_key", _P), ("sm_ent_off", _P), ("sm_ent_key", _P), ("sm_ent_val", _P)]


def _blob(items: Sequence[bytes]):
    offs = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        offs[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    return np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8).copy(), offs


def _enc(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("utf-8", "surrogateescape")


class WireBatch:
    """N CompressedAttributes messages + the global word list, in mxp_wire_batch layout."""

    def __init__(self, messages: Sequence[dict], global_words: Sequence[str]):
        self.messages = list(messages)
        self.global_words = list(global_words)
        n = self.n = len(self.messages)
        self._keep = []
        self.global_bytes, self.global_offsets = _blob([_enc(w) for w in self.global_words])
        words = [_enc(w) for m in self.messages for w in m.get("words", [])]
        self.word_bytes, self.word_offsets = _blob(words)
        self.words_off = self._off([len(m.get("words", [])) for m in self.messages])

        def field(name, vdtype, conv=lambda v: v):
            per = [sorted(m.get(name, {}).items()) for m in self.messages]
            off = self._off([len(p) for p in per])
            keys = np.array([k for p in per for k, _ in p], dtype=np.int32)
            vals = np.array([conv(v) for p in per for _, v in p], dtype=vdtype)
            return off, keys, vals, per

        self.str_off, self.str_key, self.str_val, _ = field("strings", np.int32)
        self.i64_off, self.i64_key, self.i64_val, _ = field("int64s", np.int64)
        self.dbl_off, self.dbl_key, self.dbl_val, _ = field("doubles", np.float64)
        self.bool_off, self.bool_key, self.bool_val, _ = field("bools", np.uint8, lambda v: 1 if v else 0)
        self.dur_off, self.dur_key, self.dur_val, _ = field("durations", np.int64)
        self.ts_off, self.ts_key, ts, _ = field("timestamps", np.int64, lambda v: v[0])
        self.ts_sec = ts
        self.ts_nsec = np.array([v[1] for m in self.messages for _, v in sorted(m.get("timestamps", {}).items())],
                                dtype=np.int32)
        per = [sorted(m.get("bytes", {}).items()) for m in self.messages]
        self.byt_off = self._off([len(p) for p in per])
        self.byt_key = np.array([k for p in per for k, _ in p], dtype=np.int32)
        self.byt_bytes, self.byt_val_off = _blob([bytes(v) for p in per for _, v in p])
        per = [sorted(m.get("string_maps", {}).items()) for m in self.messages]
        self.sm_off = self._off([len(p) for p in per])
        self.sm_key = np.array([k for p in per for k, _ in p], dtype=np.int32)
        ents = [sorted(v.items()) for p in per for _, v in p]
        self.sm_ent_off = self._off([len(e) for e in ents])
        self.sm_ent_key = np.array([k for e in ents for k, _ in e], dtype=np.int32)
        self.sm_ent_val = np.array([v for e in ents for _, v in e], dtype=np.int32)
        self._c = None
        assert n == len(self.words_off) - 1

    @staticmethod
    def _off(counts):
        off = np.zeros(len(counts) + 1, dtype=np.uint64)
        if counts:
            off[1:] = np.cumsum(counts, dtype=np.uint64)
        return off

    def c_struct(self) -> _CWire:
        if self._c is None:
            c = _CWire()
            c.n_requests = self.n
            c.n_global = len(self.global_words)
            for name, _ in _CWire._fields_[2:]:
                arr = getattr(self, name)
                if arr.size == 0:  # keep a valid pointer for empty arrays
                    arr = np.zeros(1, dtype=arr.dtype)
                    self._keep.append(arr)
                setattr(c, name, arr.ctypes.data)
            self._c = c
        return self._c


class WireDecoded:
    """An engine-owned mxp_wire (mxp_wire_decode); `batch()` copies it into a BagBatch."""

    def __init__(self, engine, h):
        self.engine, self.h = engine, h
        self.view = _CBatch.from_address(engine.lib.mxp_wire_view(h))
        self.n = self.view.n_requests

    def c_struct(self) -> _CBatch:
        return self.view

    def batch(self) -> BagBatch:
        v, n = self.view, self.view.n_requests

        def arr(p, count, dtype):
            if count == 0:
                return np.zeros(0, dtype=dtype)
            return np.ctypeslib.as_array(p, shape=(count,)).astype(dtype, copy=True)

        names = [v.column_names[c].decode() for c in range(v.n_columns)]
        kinds = [arr(v.kinds[c], n, np.uint8) for c in range(v.n_columns)]
        vals = [arr(v.values[c], n, np.uint64) for c in range(v.n_columns)]
        offs = arr(v.str_offsets, v.n_strings + 1, np.uint64)
        blob = arr(v.str_bytes, int(offs[-1]) + 1, np.uint8)
        moff = arr(v.map_offsets, v.n_maps + 1, np.uint64)
        return BagBatch(n, names, kinds, vals, blob, offs, arr(v.time_sec, v.n_times, np.int64),
                        arr(v.time_nsec, v.n_times, np.int32), moff, arr(v.map_keys, int(moff[-1]), np.uint32),
                        arr(v.map_values, int(moff[-1]), np.uint32))

    def __del__(self):
        if getattr(self, "h", None):
            self.engine.lib.mxp_wire_free(self.h)
            self.h = None


def decode(engine, wire: WireBatch, names: Optional[List[str]] = None) -> WireDecoded:
    h = ctypes.c_void_p()
    arr = None
    if names is not None:
        arr = (ctypes.c_char_p * max(len(names), 1))(*[_enc(x) for x in names])
    engine._check(engine.lib.mxp_wire_decode(engine.h, ctypes.byref(wire.c_struct()), arr,
                                             len(names) if names is not None else 0, ctypes.byref(h)),
                  "mxp_wire_decode")
    return WireDecoded(engine, h)


def from_bags(bags: Sequence[Dict[str, object]], global_words: Sequence[str], rng=None) -> WireBatch:
    """Encode Python bags (the BagBatch.from_bags value model: str, GoInt64, GoFloat64, bool,
    GoDuration, GoTime, bytes, dict) as CompressedAttributes the way MutableBag.ToProto does: names
    and string values from the global dictionary when present, else message words."""
    from .bags import GoDuration, GoFloat64, GoInt64, GoTime
    gdict = {w: i for i, w in enumerate(global_words)}
    msgs = []
    for b in bags:
        words: List[str] = []
        wdict: Dict[str, int] = {}

        def idx(s: str) -> int:
            if s in gdict:
                return gdict[s]
            if s not in wdict:
                wdict[s] = -len(words) - 1
                words.append(s)
            return wdict[s]

        m = {"words": words}
        for name, v in b.items():
            k = idx(name)
            if isinstance(v, bool):
                m.setdefault("bools", {})[k] = v
            elif isinstance(v, GoInt64):
                m.setdefault("int64s", {})[k] = int(v)
            elif isinstance(v, GoDuration):
                m.setdefault("durations", {})[k] = int(v)
            elif isinstance(v, GoFloat64):
                m.setdefault("doubles", {})[k] = float(v)
            elif isinstance(v, GoTime):
                m.setdefault("timestamps", {})[k] = (v.sec, v.nsec)
            elif isinstance(v, (bytes, bytearray)):
                m.setdefault("bytes", {})[k] = bytes(v)
            elif isinstance(v, dict):
                m.setdefault("string_maps", {})[k] = {idx(kk): idx(vv) for kk, vv in v.items()}
            elif isinstance(v, str):
                m.setdefault("strings", {})[k] = idx(v)
            else:
                raise TypeError("no wire form for %r" % (v,))
        msgs.append(m)
    return WireBatch(msgs, global_words)
