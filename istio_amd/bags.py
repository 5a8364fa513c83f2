"""Host-side attribute-bag batches (include/mxp_batch.h) and the Go value model they carry.

`attribute.Bag` (mixer/pkg/attribute/bag.go:18-31) hands the interpreter Go values whose *dynamic*
type matters: `resolve_s` type-asserts `string`, `resolve_i` accepts `int64` or `time.Duration`,
`ip_equal` takes `[]byte` (mixer/pkg/il/interpreter/interpreterRun.go:455-708).  Python values are
mapped to those Go types as follows:

    str                 -> string            bytes / bytearray -> []byte
    bool                -> bool              GoInt64(x) / int  -> int64
    GoFloat64(x)/float  -> float64           GoDuration(ns)    -> time.Duration
    GoTime(sec, nsec)   -> time.Time         dict[str, str]    -> map[string]string (StringMap)
    GoOther(text)       -> any other Go type (e.g. a plain Go `int`); `text` is its "%v" form

`BagBatch` lays N bags out column-wise exactly as the C-ABI expects; large synthetic batches are
built directly from numpy columns with `BagBatch.from_columns`.
"""
from __future__ import annotations

import ctypes
import struct
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

ABSENT, STRING, INT64, DOUBLE, BOOL, DURATION, TIMESTAMP, BYTES, STRING_MAP, OTHER = range(10)
KIND_NAMES = ["ABSENT", "STRING", "INT64", "DOUBLE", "BOOL", "DURATION", "TIMESTAMP", "BYTES",
              "STRING_MAP", "OTHER"]


class GoInt64(int):
    """A Go int64."""


class GoFloat64(float):
    """A Go float64."""


class GoDuration(int):
    """A Go time.Duration (nanoseconds)."""


class GoTime:
    """A Go time.Time instant (UTC seconds + nanoseconds)."""

    __slots__ = ("sec", "nsec")

    def __init__(self, sec: int, nsec: int = 0):
        self.sec = int(sec)
        self.nsec = int(nsec)

    def __eq__(self, other):  # (by name: the oracle's own GoTime compares equal too)
        return type(other).__name__ == "GoTime" and (self.sec, self.nsec) == (other.sec, other.nsec)

    def __hash__(self):
        return hash((self.sec, self.nsec))

    def __repr__(self):
        return "GoTime(%d, %d)" % (self.sec, self.nsec)


class GoOther:
    """Any other Go value (e.g. an untyped `int`); only its `%v` text is observable."""

    __slots__ = ("text",)

    def __init__(self, text: str):
        self.text = text

    def __eq__(self, other):
        return isinstance(other, GoOther) and other.text == self.text

    def __hash__(self):
        return hash(self.text)

    def __repr__(self):
        return "GoOther(%r)" % self.text


def go_str_bytes(s: str) -> bytes:
    """Go strings are byte strings; lone surrogates carry raw non-UTF-8 bytes."""
    return s.encode("utf-8", "surrogateescape")


def bytes_go_str(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def from_tagged(v):
    """Tagged JSON value (tests/golden/*.json) -> Python Go-model value."""
    t = v["t"]
    if t == "string":
        return v["v"]
    if t in ("int64",):
        return GoInt64(int(v["v"]))
    if t == "int":
        return GoOther(str(int(v["v"])))
    if t == "float64":
        return GoFloat64(float(v["v"]))
    if t == "bool":
        return bool(v["v"])
    if t == "duration":
        return GoDuration(int(v["v"]))
    if t == "time":
        return GoTime(int(v["sec"]), int(v["nsec"]))
    if t == "bytes":
        return bytes.fromhex(v["v"])
    if t == "map":
        return dict(v["v"])
    if t == "nil":
        return None
    raise ValueError("unsupported tagged value %r" % (v,))


class _CBatch(ctypes.Structure):
    _fields_ = [
        ("n_requests", ctypes.c_uint32),
        ("n_columns", ctypes.c_uint32),
        ("column_names", ctypes.POINTER(ctypes.c_char_p)),
        ("kinds", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))),
        ("values", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64))),
        ("n_strings", ctypes.c_uint32),
        ("str_bytes", ctypes.POINTER(ctypes.c_uint8)),
        ("str_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("n_times", ctypes.c_uint32),
        ("time_sec", ctypes.POINTER(ctypes.c_int64)),
        ("time_nsec", ctypes.POINTER(ctypes.c_int32)),
        ("n_maps", ctypes.c_uint32),
        ("map_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("map_keys", ctypes.POINTER(ctypes.c_uint32)),
        ("map_values", ctypes.POINTER(ctypes.c_uint32)),
    ]


def _ptr(arr, ctype):
    return arr.ctypes.data_as(ctypes.POINTER(ctype))


class StringPool:
    """Batch string table (ids are batch-local; bytes are what counts)."""

    def __init__(self):
        self.ids: Dict[bytes, int] = {}
        self.items: List[bytes] = []

    def add(self, b: bytes) -> int:
        i = self.ids.get(b)
        if i is None:
            i = len(self.items)
            self.ids[b] = i
            self.items.append(b)
        return i

    def arrays(self):
        offs = np.zeros(len(self.items) + 1, dtype=np.uint64)
        if self.items:
            offs[1:] = np.cumsum([len(x) for x in self.items], dtype=np.uint64)
        blob = np.frombuffer(b"".join(self.items) + b"\0", dtype=np.uint8).copy()
        return blob, offs


class BagBatch:
    """N attribute bags in the columnar layout of include/mxp_batch.h."""

    def __init__(self, n: int, names: Sequence[str], kinds: Sequence[np.ndarray],
                 values: Sequence[np.ndarray], str_blob: np.ndarray, str_offsets: np.ndarray,
                 time_sec: Optional[np.ndarray] = None, time_nsec: Optional[np.ndarray] = None,
                 map_offsets: Optional[np.ndarray] = None, map_keys: Optional[np.ndarray] = None,
                 map_values: Optional[np.ndarray] = None):
        self.n = int(n)
        self.names = list(names)
        self.kinds = [np.ascontiguousarray(k, dtype=np.uint8) for k in kinds]
        self.values = [np.ascontiguousarray(v, dtype=np.uint64) for v in values]
        for k, v in zip(self.kinds, self.values):
            assert k.shape == (self.n,) and v.shape == (self.n,)
        self.str_blob = np.ascontiguousarray(str_blob, dtype=np.uint8)
        if self.str_blob.size == 0:
            self.str_blob = np.zeros(1, dtype=np.uint8)
        self.str_offsets = np.ascontiguousarray(str_offsets, dtype=np.uint64)
        self.time_sec = np.ascontiguousarray(time_sec if time_sec is not None else np.zeros(0), dtype=np.int64)
        self.time_nsec = np.ascontiguousarray(time_nsec if time_nsec is not None else np.zeros(0), dtype=np.int32)
        self.map_offsets = np.ascontiguousarray(map_offsets if map_offsets is not None else np.zeros(1), dtype=np.uint64)
        self.map_keys = np.ascontiguousarray(map_keys if map_keys is not None else np.zeros(0), dtype=np.uint32)
        self.map_values = np.ascontiguousarray(map_values if map_values is not None else np.zeros(0), dtype=np.uint32)
        self._c = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_bags(cls, bags: Sequence[dict], names: Optional[Iterable[str]] = None) -> "BagBatch":
        """Build from Python dict bags (Go value model above)."""
        n = len(bags)
        if names is None:
            seen = {}
            for b in bags:
                for k in b:
                    seen.setdefault(k, None)
            names = list(seen)
        names = list(names)
        pool = StringPool()
        times_s: List[int] = []
        times_ns: List[int] = []
        map_off = [0]
        map_k: List[int] = []
        map_v: List[int] = []
        kinds = [np.zeros(n, dtype=np.uint8) for _ in names]
        values = [np.zeros(n, dtype=np.uint64) for _ in names]
        for r, bag in enumerate(bags):
            for c, name in enumerate(names):
                if name not in bag:
                    continue
                k, v = cls._encode(bag[name], pool, times_s, times_ns, map_off, map_k, map_v)
                kinds[c][r] = k
                values[c][r] = v
        blob, offs = pool.arrays()
        return cls(n, names, kinds, values, blob, offs, np.array(times_s, dtype=np.int64),
                   np.array(times_ns, dtype=np.int32), np.array(map_off, dtype=np.uint64),
                   np.array(map_k, dtype=np.uint32), np.array(map_v, dtype=np.uint32))

    @staticmethod
    def _encode(v, pool, ts, tns, moff, mk, mv):
        if isinstance(v, bool):
            return BOOL, 1 if v else 0
        if isinstance(v, GoDuration):
            return DURATION, int(v) & 0xFFFFFFFFFFFFFFFF
        if isinstance(v, (GoInt64, int)) and not isinstance(v, bool):
            return INT64, int(v) & 0xFFFFFFFFFFFFFFFF
        if isinstance(v, float):
            return DOUBLE, struct.unpack("<Q", struct.pack("<d", float(v)))[0]
        if isinstance(v, str):
            return STRING, pool.add(go_str_bytes(v))
        if isinstance(v, (bytes, bytearray)):
            return BYTES, pool.add(bytes(v))
        if isinstance(v, GoTime):
            ts.append(v.sec)
            tns.append(v.nsec)
            return TIMESTAMP, len(ts) - 1
        if isinstance(v, dict):
            for key, val in v.items():
                mk.append(pool.add(go_str_bytes(key)))
                mv.append(pool.add(go_str_bytes(val)))
            moff.append(len(mk))
            return STRING_MAP, len(moff) - 2
        if isinstance(v, GoOther):
            return OTHER, pool.add(go_str_bytes(v.text))
        raise TypeError("unsupported bag value %r" % (v,))

    @classmethod
    def from_columns(cls, n, columns: Dict[str, tuple], strings: Sequence[bytes],
                     maps: Optional[tuple] = None, times: Optional[tuple] = None) -> "BagBatch":
        """columns: name -> (kinds u8[n], values u64[n]); strings: the batch string table;
        maps: (offsets u64[M+1], keys u32[E], values u32[E]); times: (sec i64[T], nsec i32[T])."""
        offs = np.zeros(len(strings) + 1, dtype=np.uint64)
        if len(strings):
            offs[1:] = np.cumsum(np.fromiter((len(s) for s in strings), dtype=np.uint64, count=len(strings)))
        blob = np.frombuffer(b"".join(strings) + b"\0", dtype=np.uint8).copy()
        names = list(columns)
        mo, mk, mv = maps if maps is not None else (None, None, None)
        tsec, tns = times if times is not None else (None, None)
        return cls(n, names, [columns[k][0] for k in names], [columns[k][1] for k in names], blob, offs,
                   tsec, tns, mo, mk, mv)

    # ------------------------------------------------------------------ accessors
    @property
    def n_strings(self):
        return len(self.str_offsets) - 1

    def string(self, sid: int) -> bytes:
        a, b = int(self.str_offsets[sid]), int(self.str_offsets[sid + 1])
        return self.str_blob[a:b].tobytes()

    def get(self, r: int, name: str):
        """attribute.Bag.Get(name) for request r -> (value, found)."""
        if name not in self.names:
            return None, False
        c = self.names.index(name)
        k = int(self.kinds[c][r])
        v = int(self.values[c][r])
        if k == ABSENT:
            return None, False
        if k == STRING:
            return bytes_go_str(self.string(v)), True
        if k == BYTES:
            return self.string(v), True
        if k == INT64:
            return GoInt64(v - (1 << 64) if v >> 63 else v), True
        if k == DURATION:
            return GoDuration(v - (1 << 64) if v >> 63 else v), True
        if k == DOUBLE:
            return GoFloat64(struct.unpack("<d", struct.pack("<Q", v))[0]), True
        if k == BOOL:
            return bool(v), True
        if k == TIMESTAMP:
            return GoTime(int(self.time_sec[v]), int(self.time_nsec[v])), True
        if k == STRING_MAP:
            a, b = int(self.map_offsets[v]), int(self.map_offsets[v + 1])
            return {bytes_go_str(self.string(int(self.map_keys[e]))): bytes_go_str(self.string(int(self.map_values[e])))
                    for e in range(a, b)}, True
        if k == OTHER:
            return GoOther(bytes_go_str(self.string(v))), True
        raise ValueError(k)

    def subset(self, rows: np.ndarray) -> "BagBatch":
        """Rows `rows` as a new batch sharing the string/map/time tables."""
        rows = np.asarray(rows, dtype=np.int64)
        return BagBatch(len(rows), self.names, [k[rows] for k in self.kinds], [v[rows] for v in self.values],
                        self.str_blob, self.str_offsets, self.time_sec, self.time_nsec, self.map_offsets,
                        self.map_keys, self.map_values)

    # ------------------------------------------------------------------ C view
    def c_struct(self) -> _CBatch:
        if self._c is not None:
            return self._c
        nc = len(self.names)
        self._names_c = (ctypes.c_char_p * max(nc, 1))(*[n.encode() for n in self.names])
        self._kind_ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(nc, 1))(*[_ptr(k, ctypes.c_uint8) for k in self.kinds])
        self._val_ptrs = (ctypes.POINTER(ctypes.c_uint64) * max(nc, 1))(*[_ptr(v, ctypes.c_uint64) for v in self.values])
        s = _CBatch()
        s.n_requests = self.n
        s.n_columns = nc
        s.column_names = ctypes.cast(self._names_c, ctypes.POINTER(ctypes.c_char_p))
        s.kinds = ctypes.cast(self._kind_ptrs, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)))
        s.values = ctypes.cast(self._val_ptrs, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)))
        s.n_strings = self.n_strings
        s.str_bytes = _ptr(self.str_blob, ctypes.c_uint8)
        s.str_offsets = _ptr(self.str_offsets, ctypes.c_uint64)
        s.n_times = len(self.time_sec)
        s.time_sec = _ptr(self.time_sec, ctypes.c_int64)
        s.time_nsec = _ptr(self.time_nsec, ctypes.c_int32)
        s.n_maps = len(self.map_offsets) - 1
        s.map_offsets = _ptr(self.map_offsets, ctypes.c_uint64)
        s.map_keys = _ptr(self.map_keys, ctypes.c_uint32)
        s.map_values = _ptr(self.map_values, ctypes.c_uint32)
        self._c = s
        return s


class _CBatch2(ctypes.Structure):  # mxp_bag_batch2 (include/mxp_batch.h)
    _fields_ = [
        ("base", _CBatch),
        ("narrow", ctypes.POINTER(ctypes.c_uint8)),
        ("values32", ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))),
        ("str_offsets32", ctypes.POINTER(ctypes.c_uint32)),
        ("map_offsets32", ctypes.POINTER(ctypes.c_uint32)),
    ]


# kinds whose values fit 32 bits (ids, BOOL) -- a column of only these travels narrow
NARROW_KINDS = (0, 1, 4, 6, 7, 8, 9)


class NarrowBatch:
    """The narrow form of a BagBatch (mxp_bag_batch2): u32 values for the columns whose kinds are all
    id kinds or BOOL, u32 string and map offsets.  `alloc(count, dtype)` places its arrays (e.g. a
    pinned arena's `empty`); the wide columns and the other tables stay the BagBatch's own."""

    def __init__(self, batch: BagBatch, alloc=None):
        alloc = alloc or (lambda count, dtype: np.empty(count, dtype=dtype))

        def put(a, dtype):
            out = alloc(a.size, dtype)
            out[...] = a
            return out
        self.batch = batch
        ok = np.array([bool(np.isin(k, NARROW_KINDS).all()) and (v.size == 0 or int(v.max()) < (1 << 32))
                       for k, v in zip(batch.kinds, batch.values)], dtype=np.uint8)
        self.narrow = put(ok, np.uint8) if ok.size else np.zeros(1, dtype=np.uint8)
        self.values32 = [put(v, np.uint32) if f else None for v, f in zip(batch.values, ok)]
        if batch.str_offsets[-1] >= (1 << 32) or batch.map_offsets[-1] >= (1 << 32):
            raise ValueError("a narrow batch holds below 4 GiB of strings / map entries")
        self.str_offsets32 = put(batch.str_offsets, np.uint32)
        self.map_offsets32 = put(batch.map_offsets, np.uint32)
        self._c = None

    @property
    def n(self) -> int:
        return self.batch.n

    def wire_bytes(self) -> int:
        """Bytes over the link: kinds, the narrow / wide values, string bytes, u32 offsets, times, maps."""
        b = self.batch
        vals = sum(v.nbytes // 2 if f else v.nbytes for v, f in zip(b.values, self.narrow))
        return int(sum(k.nbytes for k in b.kinds) + vals + b.str_blob.nbytes + self.str_offsets32.nbytes
                   + b.time_sec.nbytes + b.time_nsec.nbytes + self.map_offsets32.nbytes + b.map_keys.nbytes
                   + b.map_values.nbytes)

    def c_struct(self) -> _CBatch2:
        if self._c is not None:
            return self._c
        b = self.batch
        s = _CBatch2()
        s.base = b.c_struct()
        s.base.str_offsets = None
        s.base.map_offsets = None
        nc = len(b.names)
        s.narrow = _ptr(self.narrow, ctypes.c_uint8)
        self._v32 = (ctypes.POINTER(ctypes.c_uint32) * max(nc, 1))(
            *[_ptr(v, ctypes.c_uint32) if v is not None else ctypes.POINTER(ctypes.c_uint32)() for v in self.values32])
        s.values32 = ctypes.cast(self._v32, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)))
        s.str_offsets32 = _ptr(self.str_offsets32, ctypes.c_uint32)
        s.map_offsets32 = _ptr(self.map_offsets32, ctypes.c_uint32)
        self._c = s
        return s
