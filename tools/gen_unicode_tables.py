"""Unicode tables for Go regexp's \\p{..} classes and (?i) case folding, generated offline.

Go 1.9's regexp/syntax reads unicode.Categories, unicode.Scripts and unicode.SimpleFold (Unicode
9.0.0).  Neither Go nor its tables are in this image, so they are rebuilt from the Unicode data this
image has: general categories from Python's unicodedata, scripts from Perl's Unicode::UCD, simple case
folding orbits from single-rune upper / lower mappings (unicodedata), all Unicode 13.0.0 here.  Runes
assigned after Unicode 9 therefore classify where Go 1.9 would not: PARITY UNPINNED (no reference
fixture covers \\p classes or non-ASCII folding).

Writes the same tables three times: the engine's C++ header, the oracle's C header and the oracle's
JSON (goregex.py).
    python tools/gen_unicode_tables.py
"""
import json
import os
import subprocess
import unicodedata

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_RUNE = 0x10FFFF

# unicode.Categories of Go 1.9 (one- and two-letter general categories)
CATEGORIES = ["C", "Cc", "Cf", "Co", "Cs", "L", "Ll", "Lm", "Lo", "Lt", "Lu", "M", "Mc", "Me", "Mn", "N", "Nd",
              "Nl", "No", "P", "Pc", "Pd", "Pe", "Pf", "Pi", "Po", "Ps", "S", "Sc", "Sk", "Sm", "So", "Z", "Zl", "Zp",
              "Zs"]


def ranges_of(pred):
    out, start = [], None
    for r in range(MAX_RUNE + 2):
        ok = r <= MAX_RUNE and pred(r)
        if ok and start is None:
            start = r
        elif not ok and start is not None:
            out.append((start, r - 1))
            start = None
    return out


def categories():
    cat = [unicodedata.category(chr(r)) for r in range(MAX_RUNE + 1)]
    out = {}
    for name in CATEGORIES:
        if len(name) == 2:
            out[name] = ranges_of(lambda r, n=name: cat[r] == n)
        elif name == "C":  # Go's C: Cc Cf Co Cs (no Cn)
            out[name] = ranges_of(lambda r: cat[r] in ("Cc", "Cf", "Co", "Cs"))
        else:
            out[name] = ranges_of(lambda r, n=name: cat[r][0] == n)
    return out


def go_script_name(perl_name):
    special = {"Signwriting": "SignWriting", "Nko": "Nko", "Phags_pa": "Phags_Pa"}
    if perl_name in special:
        return special[perl_name]
    return "_".join(p[:1].upper() + p[1:] for p in perl_name.split("_"))


def scripts():
    code = ('use Unicode::UCD; my $r = Unicode::UCD::charscripts(); for my $k (sort keys %$r) '
            '{ print $k, " ", join(" ", map { "$_->[0]-$_->[1]" } @{$r->{$k}}), "\\n"; }')
    txt = subprocess.check_output(["perl", "-e", code]).decode()
    out = {}
    for line in txt.splitlines():
        parts = line.split()
        name = go_script_name(parts[0])
        rs = sorted((int(a), int(b)) for a, b in (p.split("-") for p in parts[1:]))
        merged = []
        for a, b in rs:
            if merged and a <= merged[-1][1] + 1:
                merged[-1] = (merged[-1][0], max(merged[-1][1], b))
            else:
                merged.append((a, b))
        out[name] = merged
    out.pop("Unknown", None)
    return out


def fold_orbits():
    """Orbits of simple case folding: runes joined by their single-rune upper / lower mappings."""
    parent = list(range(MAX_RUNE + 1))

    def find(x):
        root = x
        while parent[root] != root:
            root = parent[root]
        while parent[x] != root:
            parent[x], x = root, parent[x]
        return root
    linked = set()
    for r in range(MAX_RUNE + 1):
        if 0xD800 <= r <= 0xDFFF:
            continue
        c = chr(r)
        for m in (c.lower(), c.upper()):
            if len(m) == 1 and m != c:
                a, b = find(r), find(ord(m))
                if a != b:
                    parent[max(a, b)] = min(a, b)
                linked.update((r, ord(m)))
    groups = {}
    for r in linked:
        groups.setdefault(find(r), []).append(r)
    # SimpleFold(r): the next larger rune of r's orbit, wrapping to the smallest
    nxt = []
    for g in groups.values():
        g = sorted(g)
        for i, r in enumerate(g):
            nxt.append((r, g[(i + 1) % len(g)]))
    return sorted(nxt)


def c_tables(classes, fold, banner):
    names = sorted(classes)
    lines = [banner, "#pragma once", "#include <stdint.h>", ""]
    flat, index = [], []
    for n in names:
        index.append((n, len(flat), len(classes[n])))
        flat.extend(classes[n])
    lines.append("static const uint32_t kUniRanges[%d][2] = {" % len(flat))
    for i in range(0, len(flat), 6):
        lines.append("    " + " ".join("{0x%X, 0x%X}," % r for r in flat[i:i + 6]))
    lines.append("};")
    lines.append("typedef struct { const char* name; uint32_t off, n; } uni_class;")
    lines.append("static const uni_class kUniClasses[%d] = {" % len(index))
    for n, o, k in index:
        lines.append('    {"%s", %d, %d},' % (n, o, k))
    lines.append("};")
    lines.append("/* simple case folding: {rune, next rune of its orbit} (unicode.SimpleFold), ascending */")
    lines.append("static const uint32_t kUniFold[%d][2] = {" % len(fold))
    for i in range(0, len(fold), 6):
        lines.append("    " + " ".join("{0x%X, 0x%X}," % r for r in fold[i:i + 6]))
    lines.append("};")
    return "\n".join(lines) + "\n"


def main():
    classes = categories()
    sc = scripts()
    for k, v in sc.items():
        if k not in classes:
            classes[k] = v
    fold = fold_orbits()
    note = ("Unicode %s tables for Go regexp \\\\p{..} classes (unicode.Categories + unicode.Scripts) and\n"
            " * simple case folding orbits -- generated by tools/gen_unicode_tables.py (unicodedata categories,\n"
            " * Perl Unicode::UCD scripts).  Go 1.9 reads Unicode 9.0.0 tables: PARITY UNPINNED." % unicodedata.unidata_version)
    with open(os.path.join(ROOT, "istio_amd", "csrc", "unicode_tables.h"), "w") as f:
        f.write(c_tables(classes, fold, "/* " + note + " */"))
    with open(os.path.join(ROOT, "oracle", "unicode_tables.h"), "w") as f:
        f.write(c_tables(classes, fold, "/* ORACLE (test infrastructure only) -- " + note + " */"))
    with open(os.path.join(ROOT, "oracle", "unicode_tables.json"), "w") as f:
        json.dump({"unicode": unicodedata.unidata_version, "classes": classes, "fold": fold}, f, separators=(",", ":"))
    print("classes %d, ranges %d, fold entries %d" % (len(classes), sum(len(v) for v in classes.values()), len(fold)))


if __name__ == "__main__":
    main()
