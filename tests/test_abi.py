"""The C-ABI library loads and exports every entry point include/*.h declares (no GPU needed)."""
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def declared_functions():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            names |= set(re.findall(r"^\s*(?:[A-Za-z_][A-Za-z0-9_ \*]*?[\s\*])(mxp_[a-z0-9_]+)\s*\(", src, re.M))
    return names


def test_exports_all_declared_symbols(libmxp):
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(libmxp, n)]
    assert not missing


def test_python_mirror_binds_every_symbol(libmxp):
    from istio_amd.engine import SIGNATURES
    assert declared_functions() == set(SIGNATURES)


def test_host_only_engine_refuses_eval(libmxp):
    from istio_amd.engine import Engine, MxpError
    from istio_amd.bags import BagBatch
    e = Engine(-1)
    e.set_vocabulary({"a": "INT64"})
    assert list(e.compile(["a == 2"])) == [0]
    try:
        e.eval_batch(BagBatch.from_bags([{"a": 2}]))
    except MxpError as ex:
        assert "host-only" in str(ex)
    else:
        raise AssertionError("host-only engine evaluated")


def test_gfx950_code_object(libmxp):
    data = open(os.path.join(ROOT, "istio_amd", "libmxp.so"), "rb").read()
    assert b"gfx950" in data


def test_ruleset_columns(libmxp):
    """mxp_ruleset_columns: the attributes a rule set reads (columns, then map attributes of
    map["key"] reads), then the resolver's identity and context.protocol (host-only engine)."""
    import numpy as np
    from istio_amd.engine import Engine
    eng = Engine(-1)
    assert eng.read_attributes() == []
    eng.set_vocabulary({"a": "STRING", "b": "INT64", "m": "STRING_MAP", "destination.service": "STRING",
                        "context.protocol": "STRING"})
    eng.compile(['a == "x" && b == 2', 'm["k"] == a', 'a.startsWith("y")'])
    assert eng.read_attributes() == ["a", "b", "m"]
    eng.set_resolver("destination.service", "default", ["default"] * 3, np.ones(3, np.uint32), np.zeros(3, np.uint8),
                     np.zeros(3, np.uint8))
    assert eng.read_attributes() == ["a", "b", "m", "destination.service", "context.protocol"]
