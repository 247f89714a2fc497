"""Jupyter support (flexflow_amd/jupyter.py; reference python/flexflow/jupyter.py and
jupyter_notebook/): config JSON -> FFConfig flags, kernel-spec installation."""
import json
import os

from flexflow_amd import jupyter
from flexflow_amd.config import FFConfig


def test_config_file_drives_ffconfig(tmp_path, monkeypatch):
    cfg = jupyter.default_config()
    cfg["fbmem"]["value"] = 8192
    cfg["other_options"] = [{"cmd": "-b", "value": 48}]
    p = tmp_path / "ff.json"
    p.write_text(json.dumps(cfg))
    flags = jupyter.load_jupyter_config(str(p))
    assert flags["-ll:fsize"] == 8192 and flags["-ll:gpu"] == 1 and "-ll:csize" not in flags
    monkeypatch.setattr("sys.argv", ["ipykernel_launcher", "-f", "/tmp/conn.json"])
    monkeypatch.setattr(jupyter, "_CONFIG_FILENAME", str(p))
    c = FFConfig()
    assert c.batch_size == 48


def test_install_kernel_spec(tmp_path):
    cfgfile = tmp_path / "ff.json"
    jupyter.main(["--config", str(cfgfile), "--prefix", str(tmp_path / "prefix")])
    spec = json.loads((tmp_path / "prefix" / "share" / "jupyter" / "kernels" / "flexflow_amd" / "kernel.json").read_text())
    assert spec["argv"][-2:] == ["-f", "{connection_file}"]
    assert spec["env"][jupyter.ENV_VAR] == os.path.abspath(cfgfile)
    assert json.loads(cfgfile.read_text())["gpus"]["cmd"] == "-ll:gpu"
