"""ORACLE table (test infrastructure): Go 1.9 unicode.ToUpper above ASCII, one code point at a time.

An independent derivation from the engine's range table (tools/gen_upper_table.py): candidates are the
runes whose Python full upper-casing differs from themselves (every rune with a simple uppercase
mapping is among them); for each, Perl's Unicode::UCD charinfo()->{upper} (UnicodeData.txt field 12,
the simple mapping Go's maketables reads) and charprop(Age), both kept when the rune and its capital
are assigned in Unicode 9.0.0 (Go 1.9).  Writes oracle/unicode_upper.json: [[rune, upper], ...].
    python tools/gen_oracle_upper.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cand = [r for r in range(0x80, 0x110000) if not (0xD800 <= r < 0xE000) and chr(r).upper() != chr(r)]
code = r'''use Unicode::UCD qw(charinfo charprop);
while (my $c = <STDIN>) { chomp $c; my $i = charinfo($c); my $u = $i ? $i->{upper} : "";
  my $a1 = charprop($c, "Age"); my $a2 = $u ne "" ? charprop(hex($u), "Age") : "";
  print "$c $u $a1 $a2\n"; }'''
out = subprocess.run(["perl", "-e", code], input="\n".join(map(str, cand)).encode(), stdout=subprocess.PIPE,
                     check=True).stdout.decode().splitlines()


def old(age):  # V<major>_<minor> <= V9_0
    major, minor = (int(x) for x in age[1:].split("_")[:2])
    return (major, minor) <= (9, 0)


pairs = []
for line in out:
    f = line.split()
    if len(f) < 4:
        continue
    r, u = int(f[0]), int(f[1], 16)
    if u != r and old(f[2]) and old(f[3]):
        pairs.append([r, u])
with open(os.path.join(ROOT, "oracle", "unicode_upper.json"), "w") as fh:
    json.dump({"source": "UnicodeData simple uppercase (Perl charinfo), runes and capitals assigned by 9.0.0",
               "pairs": pairs}, fh, separators=(",", ":"))
print("candidates %d, pairs %d" % (len(cand), len(pairs)), file=sys.stderr)
