"""The oracle's own Go value model (test infrastructure, not product code): the dynamic types a Go
`interface{}` result or attribute value can carry, as the restatements return them.  Kept apart from
the product's istio_amd.bags so that no product module sits on the oracle's side of a parity check;
values compare with the product's by type name and payload (GoTime by its seconds and nanoseconds),
the way ilt.AreEqual (mixer/pkg/il/testing/util.go:22-32) compares Go values."""


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

    def __eq__(self, other):
        return type(other).__name__ == "GoTime" and (self.sec, self.nsec) == (other.sec, other.nsec)

    def __hash__(self):
        return hash((self.sec, self.nsec))

    def __repr__(self):
        return "GoTime(%d, %d)" % (self.sec, self.nsec)


def go_str_bytes(s: str) -> bytes:
    """Go strings are byte strings; lone surrogates carry raw non-UTF-8 bytes."""
    return s.encode("utf-8", "surrogateescape")


def bytes_go_str(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")
