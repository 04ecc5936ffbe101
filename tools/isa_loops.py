#!/usr/bin/env python3
"""Loops (backward branches) of one kernel in a hipcc .s file, with the
instruction mix inside each.  usage: isa_loops.py FILE.s SUBSTRING [ops...]"""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
watch = sys.argv[3:] or ["v_readlane_b32", "v_writelane_b32", "ds_read_u16", "global_store_dwordx4",
                         "global_load_dwordx4", "v_alignbit_b32", "s_waitcnt", "s_setprio"]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^[_A-Za-z0-9]+:", l) and sub in l)
body = []
for l in lines[start + 1:]:
    body.append(l)
    if "s_endpgm" in l:
        break
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < i:
        seg = body[labels[tgt]:i + 1]
        ops = collections.Counter(t.split()[0] for t in (x.strip() for x in seg)
                                  if t and not t.startswith((";", ".")) and not t.endswith(":"))
        n = sum(ops.values())
        print(f"loop {tgt} lines {labels[tgt]}-{i}: {n} instrs; " +
              ", ".join(f"{w}={ops[w]}" for w in watch if ops[w]))
