"""ORACLE (test infrastructure only) -- restatement of ProtoBag.Get over CompressedAttributes.

Follows mixer/pkg/attribute/protoBag.go:
  NewProtoBag :49-65   messageDict[word i] = slotToIndex(i) = -i-1; a repeated word keeps its last slot
  Get         :91-114  getIndex fails -> not found; internalGet fails -> not found
  internalGet :161-239 Strings (lookup of the value index; error -> not found, no further probing),
                       StringMaps (lookup of every key and value; error -> not found), Int64S,
                       Doubles, Bools, Timestamps, Durations, Bytes
  getIndex    :242-252 messageDict first, then globalDict
  lookup      :255-266 index < 0 -> Words[-index-1] when defined; index >= 0 -> globalWordList[index]
and dictState.go for the index convention.  Messages are the dicts of istio_amd.wire.
"""
from __future__ import annotations

from govalue import GoDuration, GoFloat64, GoInt64, GoTime


def _lookup(msg, gwords, index):
    words = msg.get("words", [])
    if index < 0:
        slot = -index - 1
        if slot < len(words):
            return words[slot]
    elif index < len(gwords):
        return gwords[index]
    return None  # "string index %d is not defined in the available dictionaries"


def get(msg: dict, gwords, name: str):
    """ProtoBag.Get(name) -> (value, found) in the BagBatch value model."""
    mdict = {}
    for i, w in enumerate(msg.get("words", [])):
        mdict[w] = -i - 1
    gdict = {}
    for i, w in enumerate(gwords):
        gdict[w] = i
    if name in mdict:
        index = mdict[name]
    elif name in gdict:
        index = gdict[name]
    else:
        return None, False
    if index in msg.get("strings", {}):
        s = _lookup(msg, gwords, msg["strings"][index])
        return (s, True) if s is not None else (None, False)
    if index in msg.get("string_maps", {}):
        out = {}
        for k, v in msg["string_maps"][index].items():
            ks, vs = _lookup(msg, gwords, k), _lookup(msg, gwords, v)
            if ks is None or vs is None:
                return None, False
            out[ks] = vs
        return out, True
    if index in msg.get("int64s", {}):
        return GoInt64(msg["int64s"][index]), True
    if index in msg.get("doubles", {}):
        return GoFloat64(msg["doubles"][index]), True
    if index in msg.get("bools", {}):
        return bool(msg["bools"][index]), True
    if index in msg.get("timestamps", {}):
        sec, nsec = msg["timestamps"][index]
        return GoTime(sec, nsec), True
    if index in msg.get("durations", {}):
        return GoDuration(msg["durations"][index]), True
    if index in msg.get("bytes", {}):
        return bytes(msg["bytes"][index]), True
    return None, False
