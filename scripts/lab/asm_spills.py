#!/usr/bin/env python3
"""Spill report of the kernels in a device .s file (hipcc --cuda-device-only -S): per kernel whose
name contains the substring, the scratch loads / stores in total and inside loop bodies (basic
blocks LLVM annotates 'in Loop' / 'Loop Header').
usage: asm_spills.py file.s [name_substring] [-v]"""
import re
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-v" else ""
verbose = "-v" in sys.argv
lines = open(src).read().split("\n")
starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l.split(":")[0]]
for start in starts:
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    in_loop = False
    n_loop = n_all = mfma = 0
    for l in lines[start:end]:
        if re.match(r"^(\.LBB|; %bb)", l):
            in_loop = "in Loop" in l or "Loop Header" in l
        if "scratch_" in l:
            n_all += 1
            if in_loop:
                n_loop += 1
                if verbose:
                    print("  loop:", l.strip()[:100])
        if "v_mfma" in l and in_loop:
            mfma += 1
    name = lines[start].split(':')[0][:90]
    print(f"{name}: scratch ops {n_all} ({n_loop} in loops), loop MFMAs {mfma}")
