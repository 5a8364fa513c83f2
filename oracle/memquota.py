"""ORACLE (test infrastructure only) -- restatement of Mixer's memquota adapter.

  rollingWindow  mixer/adapter/memquota/rollingWindow.go:21-113 (alloc, release, roll, available)
  alloc / free   mixer/adapter/memquota/memquota.go:119-214 (cells for ValidDuration 0, rolling
                 windows of ceil(ValidDuration / 1s) * ticksPerSecond ticks otherwise; best effort
                 grabs what is left; a free of an absent cell / window returns 0)
  HandleQuota    memquota.go:107-117 (amount > 0 alloc, < 0 free, 0 nothing)
  ticks          dedup.go:51-55 (ticksPerSecond 10, currentTick = UnixNano / nanosPerTick)
  Dedup          dedup.go:58-95 handleDedup: a DeduplicationID seen before returns its first amount
                 (kept by the CALLER of the engine, restated here for the reference test table).
"""
from __future__ import annotations

TICKS_PER_SECOND = 10
NANOS_PER_TICK = 10**9 // TICKS_PER_SECOND


class RollingWindow:
    def __init__(self, limit, ticks):
        self.avail = limit
        self.slots = [0] * ticks
        self.cur = 0
        self.cur_tick = 0

    def roll(self, tick):
        behind = tick - self.cur_tick
        if behind > len(self.slots):
            behind = len(self.slots)
        for i in range(behind):
            idx = (self.cur + 1 + i) % len(self.slots)
            self.avail += self.slots[idx]
            self.slots[idx] = 0
        self.cur = (self.cur + behind) % len(self.slots)
        self.cur_tick = tick

    def alloc(self, amount, tick):
        self.roll(tick)
        if amount > self.avail:
            return False
        self.slots[self.cur] += amount
        self.avail -= amount
        return True

    def release(self, amount, tick):
        self.roll(tick)
        total, idx = 0, self.cur
        for _ in range(len(self.slots)):
            av = self.slots[idx]
            if av >= amount:
                self.slots[idx] -= amount
                total += amount
                break
            self.slots[idx] = 0
            total += av
            amount -= av
            idx -= 1
            if idx < 0:
                idx = len(self.slots) - 1
        self.avail += total
        return total


class Memquota:
    """limits: key -> (max_amount, valid_duration_ns)."""

    def __init__(self, limits):
        self.limits = dict(limits)
        self.cells, self.windows = {}, {}

    def handle(self, key, amount, best_effort, now_ns):
        if amount > 0:
            return self.alloc(key, amount, best_effort, now_ns)
        if amount < 0:
            return self.free(key, -amount, now_ns)
        return 0

    def alloc(self, key, amount, best_effort, now_ns):
        mx, vd = self.limits[key]
        tick = now_ns // NANOS_PER_TICK
        result = amount
        if vd == 0:
            in_use = self.cells.get(key, 0)
            if result > mx - in_use:
                if not best_effort:
                    return 0
                result = mx - in_use
            self.cells[key] = in_use + result
            return result
        w = self.windows.get(key)
        if w is None:
            seconds = (vd + 10**9 - 1) // 10**9
            w = self.windows[key] = RollingWindow(mx, seconds * TICKS_PER_SECOND)
        if not w.alloc(result, tick):
            if not best_effort:
                return 0
            result = w.avail
            w.alloc(result, tick)
        return result

    def free(self, key, amount, now_ns):
        mx, vd = self.limits[key]
        tick = now_ns // NANOS_PER_TICK
        if vd == 0:
            in_use = self.cells.get(key, 0)
            if amount >= in_use:
                self.cells.pop(key, None)
                return in_use
            self.cells[key] = in_use - amount
            return amount
        w = self.windows.get(key)
        if w is None:
            return 0
        result = w.release(amount, tick)
        if w.avail == mx:
            del self.windows[key]
        return result


class Dedup:
    """handleDedup's effect within one test: a repeated id returns its first amount."""

    def __init__(self):
        self.seen = {}

    def __call__(self, dedup_id, fn):
        if dedup_id in self.seen:
            return self.seen[dedup_id]
        r = fn()
        self.seen[dedup_id] = r
        return r


class CMemquota:
    """The C restatement (memquota_oracle.c, liboracle.so): the same semantics for keys 0 .. K-1
    (limits: arrays of max_amount and valid_duration_ns), a batch at a time, keys handled in
    parallel on `threads` host threads.  The bench's CPU baseline; checked against Memquota."""

    def __init__(self, max_amount, valid_ns):
        import ctypes
        import numpy as np
        import oracle
        self._L = oracle.lib()
        mx = np.ascontiguousarray(max_amount, dtype=np.int64)
        vd = np.ascontiguousarray(valid_ns, dtype=np.int64)
        self.n_keys = len(mx)
        self._h = self._L.mq_create(len(mx), mx.ctypes.data, vd.ctypes.data)
        if not self._h:
            raise MemoryError("mq_create")
        self._ct = ctypes

    def handle_batch(self, keys, amounts, best_effort, now_ns, threads=1):
        import numpy as np
        k = np.ascontiguousarray(keys, dtype=np.int32)
        a = np.ascontiguousarray(amounts, dtype=np.int64)
        b = np.ascontiguousarray(best_effort, dtype=np.uint8)
        g = np.zeros(len(k), dtype=np.int64)
        rc = self._L.mq_handle_batch(self._h, len(k), k.ctypes.data, a.ctypes.data, b.ctypes.data, int(now_ns),
                                     g.ctypes.data, int(threads))
        if rc:
            raise MemoryError("mq_handle_batch")
        return g

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.mq_destroy(self._h)
            self._h = None
