"""net.ParseIP beyond the reference's rows, corroborated against Python's `ipaddress` on the syntax
the two agree on (what test_regex_vs_python_re.py does for regexps): dotted-quad IPv4 without leading
zeros, IPv6 in full, compressed and IPv4-embedded forms, and malformed variants of both.  Go 1.9's
parseIPv4 accepts leading zeros and Python 3.10 rejects them, and Python accepts IPv6 scope ids
(`%eth0`) that Go's ParseIP rejects: both are left out of the comparison (corroboration, not
pinning -- `ipaddress` is not Go's net package).

CPU: the oracle's restatement (oracle/goval.c oracle_parse_ip).  GPU: the product's CIDR list
(netparse.h on the device, mxp_list_check) against ipaddress membership on the same strings."""
import ctypes
import ipaddress
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))


def _py_parse(s: str):
    """16-byte form as Go's ParseIP returns it (IPv4 as ::ffff:a.b.c.d), or None."""
    try:
        a = ipaddress.ip_address(s)
    except ValueError:
        return None
    if isinstance(a, ipaddress.IPv4Address):
        return b"\0" * 10 + b"\xff\xff" + a.packed
    return a.packed


def _strings(seed=7, n=6000):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.3:  # IPv4, no leading zeros
            out.append(".".join(str(int(x)) for x in rng.integers(0, 256, 4)))
        elif r < 0.6:  # IPv6 full / compressed
            g = ["%x" % int(x) for x in rng.integers(0, 1 << 16, 8)]
            if rng.random() < 0.6:
                a = int(rng.integers(0, 8))
                b = int(rng.integers(a, 9))
                s = ":".join(g[:a]) + "::" + ":".join(g[b:])
            else:
                s = ":".join(g)
            out.append(s)
        elif r < 0.7:  # IPv6 with an embedded IPv4 tail
            g = ["%x" % int(x) for x in rng.integers(0, 1 << 16, 6)]
            v4 = ".".join(str(int(x)) for x in rng.integers(0, 256, 4))
            pre = ":".join(g[: int(rng.integers(0, 6))])
            out.append(("::ffff:" if rng.random() < 0.5 else pre + "::") + v4)
        else:  # malformed variants
            base = out[int(rng.integers(0, len(out)))] if out else "1.2.3.4"
            k = int(rng.integers(0, 9))
            if k == 0:
                s = base + "."
            elif k == 1:
                s = base.replace(".", "..", 1) if "." in base else base + ":::"
            elif k == 2:
                s = "256." + base
            elif k == 3:
                s = base + ":1ffff"
            elif k == 4:
                s = " " + base
            elif k == 5:
                s = base[:-1]
            elif k == 6:
                s = base.replace(":", "", 1)
            elif k == 7:
                s = "1.2.3.4.5"
            else:
                s = "::1::2"
            out.append(s)
    # (the known divergences are left out: leading zeros in a dotted quad, scope ids)
    def leading_zero(s):
        return any(len(p) > 1 and p[0] == "0" and p.isdigit() for p in s.replace(":", ".").split("."))
    return [s for s in out if "%" not in s and not leading_zero(s)]


def test_oracle_parse_ip_agrees_with_ipaddress():
    import oracle
    L = oracle.lib()
    L.oracle_parse_ip.restype = ctypes.c_int
    L.oracle_parse_ip.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
    strs = _strings()
    valid = 0
    for s in strs:
        b = s.encode()
        buf = ctypes.create_string_buffer(16)
        ok = L.oracle_parse_ip(b, len(b), buf)
        want = _py_parse(s)
        assert bool(ok) == (want is not None), s
        if want is not None:
            assert buf.raw == want, s
            valid += 1
    assert valid > 2000 and len(strs) - valid > 500


@pytest.mark.gpu
def test_device_ip_list_agrees_with_ipaddress(libmxp):
    """The product's CIDR list (device ParseIP + interval search, HandleListEntry codes) against
    ipaddress membership on the same strings."""
    import istio_amd.engine as mxp
    import lists as L
    rng = np.random.default_rng(9)
    nets4 = ["%d.%d.0.0/%d" % (int(a), int(b), int(p)) for a, b, p in zip(rng.integers(1, 223, 300),
                                                                       rng.integers(0, 256, 300), rng.integers(8, 25, 300))]
    nets6 = ["%x:%x::/%d" % (int(a), int(b), int(p)) for a, b, p in zip(rng.integers(0x2000, 0x3fff, 200),
                                                                     rng.integers(0, 1 << 16, 200), rng.integers(16, 33, 200))]
    nets = [ipaddress.ip_network(n, strict=False) for n in nets4 + nets6]
    strs = _strings(seed=11, n=20000)
    for n in nets[:400]:  # (symbols inside listed networks too)
        strs.append(str(n.network_address + int(rng.integers(0, min(n.num_addresses, 1 << 16)))))
    eng = mxp.Engine(0)
    lst = eng.list_create(L.IP_ADDRESSES, [str(n) for n in nets], [])
    got = lst.check(strs)
    want = []
    for s in strs:
        try:
            a = ipaddress.ip_address(s)
        except ValueError:
            want.append(L.INVALID_ARGUMENT)
            continue
        if isinstance(a, ipaddress.IPv6Address) and a.ipv4_mapped is not None:
            a = a.ipv4_mapped  # (Go: a v4-in-v6 address is the IPv4 address)
        hit = any(a.version == n.version and a in n for n in nets)
        want.append(L.OK if hit else L.NOT_FOUND)
    want = np.array(want, dtype=np.int32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(strs[i], int(got[i]), int(want[i])) for i in bad[:8]]
    assert (want == L.OK).sum() > 300 and (want == L.INVALID_ARGUMENT).sum() > 500
    eng.close()
