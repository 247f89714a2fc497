"""Jupyter support (reference python/flexflow/jupyter.py + jupyter_notebook/): a notebook cannot pass
FlexFlow flags on a command line, so a JSON file maps machine settings to flags and FFConfig()
picks them up when no argv is given.

    from flexflow_amd import jupyter
    jupyter.set_jupyter_config("flexflow_jupyter.json")
    cfg = FFConfig()            # -ll:gpu / -ll:fsize / ... from the file

The file format is the reference's (`{"gpus": {"cmd": "-ll:gpu", "value": 1}, ...}`); keys with a
null value are skipped and `other_options` entries are appended. `install_kernel` writes a Jupyter
kernel spec that starts an ipykernel with the config file exported (no jupyter_client needed:
a kernel spec is one kernel.json in <prefix>/share/jupyter/kernels/<name>/).
"""
from __future__ import annotations

import json
import os
import sys

_CONFIG_FILENAME: str | None = None
ENV_VAR = "FF_JUPYTER_CONFIG"
_KEYS = ["cpus", "gpus", "utility", "sysmem", "fbmem", "zcmem", "regmem", "nodes", "ranks_per_node"]


def set_jupyter_config(filename: str) -> None:
    global _CONFIG_FILENAME
    _CONFIG_FILENAME = filename
    print("config file is set to:", filename)


def config_filename() -> str | None:
    return _CONFIG_FILENAME or os.environ.get(ENV_VAR)


def load_jupyter_config(filename: str | None = None) -> dict:
    """{flag: value} from the config file (reference load_jupyter_config)."""
    filename = filename or config_filename()
    if filename is None:
        raise RuntimeError("jupyter configuration file is not set: call set_jupyter_config(path)")
    with open(filename) as f:
        cfg = json.load(f)
    out = {}
    for k in _KEYS:
        ent = cfg.get(k)
        if isinstance(ent, dict) and ent.get("value") is not None:
            out[ent["cmd"]] = ent["value"]
    for ent in cfg.get("other_options") or []:
        if ent.get("value") is not None:
            out[ent["cmd"]] = ent["value"]
    return out


def jupyter_argv(filename: str | None = None) -> list[str]:
    """The config as an argv list for FFConfig.parse_args ([] when no file is set)."""
    if config_filename() is None and filename is None:
        return []
    argv = []
    for k, v in load_jupyter_config(filename).items():
        argv += [k] if v is True else [k, str(v)]
    return argv


def default_config() -> dict:
    """A single-GPU config in the reference's format (jupyter_notebook/flexflow_jupyter.json)."""
    ent = lambda cmd, v: {"cmd": cmd, "value": v}  # noqa: E731
    return {"name": "FlexFlow-AMD", "kernel_name": "flexflow_amd", "cpus": ent("-ll:cpu", 1),
            "gpus": ent("-ll:gpu", 1), "utility": ent("-ll:util", 1), "sysmem": ent("-ll:csize", None),
            "fbmem": ent("-ll:fsize", 4096), "zcmem": ent("-ll:zsize", 10240), "regmem": ent("-ll:rsize", None),
            "other_options": []}


def install_kernel(config_file: str, prefix: str | None = None, name: str = "flexflow_amd",
                   display_name: str = "FlexFlow-AMD (MI355X)") -> str:
    """Write <prefix>/share/jupyter/kernels/<name>/kernel.json (prefix defaults to the user data
    dir ~/.local); the kernel runs ipykernel under this interpreter with FF_JUPYTER_CONFIG set."""
    base = os.path.join(prefix, "share", "jupyter", "kernels") if prefix else \
        os.path.join(os.path.expanduser("~"), ".local", "share", "jupyter", "kernels")
    d = os.path.join(base, name)
    os.makedirs(d, exist_ok=True)
    spec = {"argv": [sys.executable, "-m", "ipykernel_launcher", "-f", "{connection_file}"],
            "display_name": display_name, "language": "python",
            "env": {ENV_VAR: os.path.abspath(config_file), "HSA_ENABLE_IPC_MODE_LEGACY": "0"}}
    with open(os.path.join(d, "kernel.json"), "w") as f:
        json.dump(spec, f, indent=1, sort_keys=True)
    return d


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="python -m flexflow_amd.jupyter", description=install_kernel.__doc__)
    ap.add_argument("--config", help="config JSON (written with defaults when missing)",
                    default="flexflow_jupyter.json")
    ap.add_argument("--prefix", default=None)
    ap.add_argument("--name", default="flexflow_amd")
    a = ap.parse_args(argv)
    if not os.path.exists(a.config):
        with open(a.config, "w") as f:
            json.dump(default_config(), f, indent=1)
    print("installed kernel spec in", install_kernel(a.config, a.prefix, a.name))


if __name__ == "__main__":
    main()
