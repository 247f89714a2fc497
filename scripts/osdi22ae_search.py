#!/usr/bin/env python3
"""Joint Unity search rehearsals at the reference's own Unity configurations
(/root/reference/scripts/osdi22ae/*.sh: every model at -ll:gpu 4 with its --budget and -b), here at
N = 4 and N = 8 devices, in ONE process planning for N devices on the analytic MI355X cost model
(or measured op costs on a GPU box).

For every (model, N) it writes profiles/search_<model>_<N>dev_r4.json (strategy + search report:
accepted rewrites, predicted ms, predicted speedup vs data parallel, the rewrites tried) and one
summary line to stdout / the summary file, including the op classes the plan does NOT run data
parallel, or — when DP wins — the cheapest rejected rewrite per family (why DP wins).

usage: osdi22ae_search.py [out_dir=profiles] [models=all] [devices=4,8]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (model, global batch, --budget) as in scripts/osdi22ae/*.sh; the reference's default -b is 64
RUNS = [("transformer", 8, 30), ("bert-large", 8, 30), ("inception_v3", 64, 10), ("dlrm", 64, 20),
        ("candle_uno", 64, 20), ("mlp_unify", 64, 20), ("xdl", 64, 20), ("resnext50", 16, 20)]


def summarize(path, model, n, batch, wall):
    d = json.load(open(path))
    ops = d.get("ops", {})
    non_dp = {}
    for name, c in ops.items():
        degs = c["degrees"]
        if any(x > 1 for x in degs[1:]) or len(set(c["devices"])) not in (1, n) or (degs and degs[0] not in (1, n)):
            non_dp[tuple(degs)] = non_dp.get(tuple(degs), 0) + 1
    single = sum(1 for c in ops.values() if len(set(c["devices"])) == 1)
    best_rej = {}
    for t in d.get("tried", []):
        fam = t["xfer"].split("[")[0]
        if fam not in best_rej or t["predicted_ms"] < best_rej[fam]:
            best_rej[fam] = t["predicted_ms"]
    return {"model": model, "devices": n, "batch": batch, "predicted_ms": d.get("predicted_ms"),
            "predicted_dp_ms": d.get("predicted_dp_ms"), "speedup_vs_dp": d.get("predicted_speedup_vs_dp"),
            "rewrites": [r["xfer"] for r in d.get("rewrites", [])], "graphs_costed": d.get("graphs_costed"),
            "graphs_popped": d.get("graphs_popped"), "non_dp_degree_vectors": {str(k): v for k, v in non_dp.items()},
            "ops_on_one_device": single, "ops": len(ops),
            "nonsequence_splits_accepted": sum(1 for s in d.get("nonsequence_splits", []) if s.get("accepted")),
            "best_tried_ms_per_family": dict(sorted(best_rej.items(), key=lambda kv: kv[1])[:8]),
            "wall_s": round(wall, 1)}


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles")
    models = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] != "all" else [r[0] for r in RUNS]
    devs = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "4,8").split(",")]
    os.makedirs(out_dir, exist_ok=True)
    lines = []
    for model, batch, budget in RUNS:
        if model not in models:
            continue
        for n in devs:
            path = os.path.join(out_dir, f"search_{model}_{n}dev_r4.json")
            t0 = time.time()
            r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "export_search.py"), model, str(n), path,
                                "unity", str(batch), "--budget", str(budget)], capture_output=True, text=True)
            if r.returncode != 0:
                print(f"{model} N={n}: FAILED\n{r.stderr[-2000:]}", flush=True)
                continue
            s = summarize(path, model, n, batch, time.time() - t0)
            lines.append(s)
            print(json.dumps(s), flush=True)
    with open(os.path.join(out_dir, "search_osdi22ae_r4.jsonl"), "w") as f:
        for s in lines:
            f.write(json.dumps(s) + "\n")


if __name__ == "__main__":
    main()
