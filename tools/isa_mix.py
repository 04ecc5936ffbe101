#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc --save-temps .s file.

usage: isa_mix.py FILE.s SUBSTRING   (first kernel whose symbol contains SUBSTRING)
Prints VGPR/SGPR counts and per-opcode counts of the static code (not a
dynamic count: loops count once)."""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^[_A-Za-z0-9]+:", l) and sub in l and not l.startswith("."))
name = lines[start].split(":")[0]
body = []
for l in lines[start + 1:]:
    if "s_endpgm" in l:
        break
    body.append(l)
ops = collections.Counter()
for l in body:
    t = l.strip()
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    ops[t.split()[0]] += 1
print(name)
for l in lines:
    if l.startswith(".set " + name + ".num_vgpr") or l.startswith(".set " + name + ".numbered_sgpr"):
        print(l)
for k, v in ops.most_common():
    print("%6d %s" % (v, k))
