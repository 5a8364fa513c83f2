"""Unicode tables for Go regexp's \\p{..} classes and (?i) case folding, generated offline.

Go 1.9's regexp/syntax reads unicode.Categories, unicode.Scripts and unicode.SimpleFold (Unicode
9.0.0).  Neither Go nor its tables are in this image, so they are rebuilt from the Unicode data this
image has (13.0.0) cut back to Unicode 9.0.0 by each code point's Age (Perl Unicode::UCD
prop_invmap("Age")): a rune assigned after 9.0 is unassigned (Cn, no script, no fold), as in Go 1.9.
  * general categories: Python's unicodedata;
  * scripts: Perl Unicode::UCD charscripts;
  * simple case folding orbits: the runes sharing one Simple_Case_Folding target (CaseFolding.txt
    statuses C + S, Perl prop_invmap), as Go's maketables groups them -- so a rune with upper / lower
    mappings but no C/S folding (U+0130, U+0131) folds only to itself, as in Go's caseOrbit.
Category or script changes of already-assigned runes between 9.0 and 13.0 are not undone: PARITY
UNPINNED (no reference fixture covers \\p classes or non-ASCII folding).

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


GO_UNICODE = (9, 0)  # Go 1.9's unicode package: Unicode 9.0.0


def invmap(prop):
    """Perl Unicode::UCD prop_invmap(prop): (range starts, values, format)."""
    code = ('use Unicode::UCD; my ($l, $m, $f, $d) = Unicode::UCD::prop_invmap("%s"); print "$f\\n"; '
            'for my $i (0 .. $#$l) { my $v = $m->[$i]; $v = join(",", @$v) if ref $v; print "$l->[$i] $v\\n"; }' % prop)
    lines = subprocess.check_output(["perl", "-e", code]).decode().splitlines()
    starts, vals = [], []
    for line in lines[1:]:
        a, _, b = line.partition(" ")
        starts.append(int(a))
        vals.append(b)
    return starts, vals, lines[0]


def go_assigned():
    """assigned[r]: r exists in Unicode 9.0 (Age <= 9.0)."""
    starts, vals, _ = invmap("Age")
    out = bytearray(MAX_RUNE + 1)
    for i, a in enumerate(starts):
        b = starts[i + 1] if i + 1 < len(starts) else MAX_RUNE + 1
        v = vals[i]
        if v == "Unassigned":
            continue
        major, minor = (int(x) for x in v.split(".")[:2])
        if (major, minor) <= GO_UNICODE:
            out[a:b] = b"\x01" * (b - a)
    return out


ASSIGNED = None


def assigned(r):
    global ASSIGNED
    if ASSIGNED is None:
        ASSIGNED = go_assigned()
    return ASSIGNED[r] == 1


def categories():
    cat = [unicodedata.category(chr(r)) if assigned(r) else "Cn" for r in range(MAX_RUNE + 1)]
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
        out[name] = [rg for a, b in merged for rg in ranges_within(a, b)]
    out.pop("Unknown", None)
    return {k: v for k, v in out.items() if v}


def ranges_within(a, b):
    """[a, b] cut to the runes assigned in Unicode 9.0."""
    out, start = [], None
    for r in range(a, b + 2):
        ok = r <= b and assigned(r)
        if ok and start is None:
            start = r
        elif not ok and start is not None:
            out.append((start, r - 1))
            start = None
    return out


def fold_orbits():
    """unicode.SimpleFold orbits: each Simple_Case_Folding target with the runes that fold to it
    (CaseFolding.txt C + S; Go maketables caseGroups), Unicode 9.0 runes only.  Returns the
    (rune, next rune of its orbit) pairs, the largest wrapping to the smallest."""
    starts, vals, fmt = invmap("Simple_Case_Folding")
    assert fmt.startswith("a"), fmt  # adjusted: a range's value grows with the code point; 0 = itself
    groups = {}
    for i, a in enumerate(starts):
        b = starts[i + 1] if i + 1 < len(starts) else MAX_RUNE + 1
        v = int(vals[i])
        if v == 0:
            continue
        for r in range(a, b):
            t = v + (r - a)
            if t != r and assigned(r) and assigned(t):
                groups.setdefault(t, {t}).add(r)
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
    note = ("Unicode 9.0.0 (Go 1.9) tables for Go regexp \\\\p{..} classes (unicode.Categories +\n"
            " * unicode.Scripts) and simple case folding orbits -- generated by tools/gen_unicode_tables.py\n"
            " * from the image's Unicode %s data cut to Age <= 9.0 (unicodedata categories, Perl\n"
            " * Unicode::UCD scripts and Simple_Case_Folding).  PARITY UNPINNED." % unicodedata.unidata_version)
    with open(os.path.join(ROOT, "istio_amd", "csrc", "unicode_tables.h"), "w") as f:
        f.write(c_tables(classes, fold, "/* " + note + " */"))
    with open(os.path.join(ROOT, "oracle", "unicode_tables.h"), "w") as f:
        f.write(c_tables(classes, fold, "/* ORACLE (test infrastructure only) -- " + note + " */"))
    with open(os.path.join(ROOT, "oracle", "unicode_tables.json"), "w") as f:
        json.dump({"unicode": "9.0.0 (cut from %s by Age)" % unicodedata.unidata_version, "classes": classes, "fold": fold}, f, separators=(",", ":"))
    print("classes %d, ranges %d, fold entries %d" % (len(classes), sum(len(v) for v in classes.values()), len(fold)))


if __name__ == "__main__":
    main()
