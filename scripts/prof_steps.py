#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV.

Steps are delimited by the optimizer kernel (one fused adam/sgd launch per weight arena per step);
the first `--skip` steps (autotuning, graph capture warm-up) are dropped so the numbers reflect
the steady state only. With the overlapped update (one optimizer launch per gradient bucket, on a
side stream) delimit steps by a once-per-step kernel instead, e.g. `--delim softmax_xent_kernel`;
busy then exceeds span by the overlapped time.  Prints ms/step per kernel (grouped by demangled-name prefix), the busy
time and the wall span per step (span - busy = launch gaps / host stalls).

usage: prof_steps.py run_kernel_trace.csv [--skip 2] [--top 40] [--delim adam_kernel]
"""
import argparse
import csv
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip", type=int, default=2)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--delim", default=None,
                help="regex of a once-per-step kernel (default: the optimizer kernel, or softmax_xent_kernel "
                     "when the optimizer runs once per gradient bucket)")
a = ap.parse_args()

rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if a.delim is None:
    n_opt = sum(1 for r in rows if re.search("adam_kernel|sgd_kernel", r["Kernel_Name"]))
    n_xent = sum(1 for r in rows if "softmax_xent_kernel" in r["Kernel_Name"])
    a.delim = "softmax_xent_kernel" if n_xent and n_opt > n_xent else "adam_kernel|sgd_kernel"
delim = re.compile(a.delim)
ends = [i for i, r in enumerate(rows) if delim.search(r["Kernel_Name"])]
# several arenas -> several optimizer launches back to back; keep the last of each run
marks = [e for k, e in enumerate(ends) if k + 1 == len(ends) or ends[k + 1] != e + 1]
if len(marks) <= a.skip + 1:
    raise SystemExit(f"only {len(marks)} steps found")
lo, hi = marks[a.skip] + 1, marks[-1] + 1
steps = len(marks) - 1 - a.skip
win = rows[lo:hi]
per = defaultdict(lambda: [0.0, 0])


def short(n):
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"^void ", "", n)
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        m = re.search(r"MT\d+x\d+x\d+", n)
        return "hipblaslt " + n.split("_")[1 if n.startswith("Cijk") else 2] + "_" + \
            n.split("_")[2 if n.startswith("Cijk") else 3] + " " + (m.group(0) if m else "")
    return n[:110]


busy = 0.0
for r in win:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    k = short(r["Kernel_Name"])
    per[k][0] += d
    per[k][1] += 1
    busy += d
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6
print(f"{steps} steps: busy {busy / steps:.3f} ms/step, span {span / steps:.3f} ms/step, "
      f"{len(win) / steps:.0f} kernels/step")
for k, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
    print(f"{t / steps:8.3f} ms/step {c / steps:6.1f}/step {100 * t / busy:5.1f}%  {k}")
