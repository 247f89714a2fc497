#!/usr/bin/env python3
"""Merge TunableOp result tables (same Validator header) into one: merge_tunable.py OUT IN...
Later files win for a repeated (op, shape) key."""
import sys

out, ins = sys.argv[1], sys.argv[2:]
header, rows = [], {}
for p in ins:
    for line in open(p).read().splitlines():
        f = line.split(",")
        if f[0] == "Validator":
            if line not in header:
                header.append(line)
        elif len(f) >= 3:
            rows[(f[0], f[1])] = line
with open(out, "w") as fo:
    fo.write("\n".join(header + [rows[k] for k in sorted(rows)]) + "\n")
print(f"{out}: {len(rows)} entries from {len(ins)} tables")
