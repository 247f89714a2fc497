"""`python -m flexflow_amd.run [--nproc N] script.py [args...]` — the job launcher (reference
src/runtime/cpp_driver.cc + the `flexflow_python` / mpirun wrappers; SURVEY R21 'ffrun').

One process per GPU on one node (the SPMD model of this framework): a thin front end over
torch.distributed.run that fills in what FlexFlow users expect — N defaults to every visible GPU,
rendezvous on 127.0.0.1, `-ll:gpu N` / `--nproc-per-node N` accepted — and keeps the RCCL/HSA
environment the pool needs (HSA_ENABLE_IPC_MODE_LEGACY=0 for dmabuf IPC). Multi-node jobs pass
--nnodes/--node-rank/--master-addr through unchanged.
"""
from __future__ import annotations

import os
import sys


def _gpu_count() -> int:
    try:
        import torch
        return max(1, torch.cuda.device_count())  # does not initialise the GPU on this image
    except Exception:  # noqa: BLE001
        return 1


def build_argv(argv):
    nproc = None
    passthrough = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("--nproc", "--nproc-per-node", "--nproc_per_node", "-ll:gpu"):
            nproc = int(argv[i + 1])
            i += 2
            continue
        if a.startswith("--nproc-per-node=") or a.startswith("--nproc="):
            nproc = int(a.split("=", 1)[1])
            i += 1
            continue
        if not a.startswith("-"):
            passthrough += argv[i:]
            break
        passthrough.append(a)
        i += 1
    launcher = ["--nproc-per-node", str(nproc or _gpu_count())]
    if not any(p.startswith("--master-addr") or p.startswith("--master_addr") or p.startswith("--rdzv")
               for p in passthrough):
        launcher += ["--master-addr", "127.0.0.1"]
    if not any(p.startswith("--master-port") or p.startswith("--master_port") for p in passthrough):
        launcher += ["--master-port", str(29500 + os.getpid() % 1000)]
    if not any(p.startswith("--nnodes") for p in passthrough):
        launcher += ["--nnodes", "1"]
    return launcher + passthrough


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from torch.distributed.run import main as tr_main
    return tr_main(build_argv(argv))


if __name__ == "__main__":
    sys.exit(main())
