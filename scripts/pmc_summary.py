#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter CSVs per kernel (name filter), print per-dispatch means."""
import csv
import re
import sys
from collections import defaultdict

pat = re.compile(sys.argv[1])
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if not pat.search(n):
            continue
        k = re.sub(r"\(.*$", "", n)[:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add((path, r["Dispatch_Id"]))
for k, d in acc.items():
    nd = len(cnt[k]) / max(1, len({p for p, _ in cnt[k]}))
    print(f"== {k}  (dispatches/file {nd:.0f})")
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {v / max(1, len(cnt[k])):.4g}")
    w = d.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in d:
                print(f"   {c}/WAVE_CYCLES = {d[c] / w:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
        print(f"   MFMA busy / (GUI_ACTIVE*CUs*4?) raw ratio = {d['SQ_VALU_MFMA_BUSY_CYCLES'] / d['GRBM_GUI_ACTIVE']:.2f}")
