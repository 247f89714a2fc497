"""C API (csrc/capi/flexflow_c.h): a C program builds, trains and queries an MLP through
libflexflow_c.so (embedded CPython driving flexflow_amd)."""
import os
import subprocess
import sys
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_program_trains_mlp(tmp_path):
    lib = os.path.join(ROOT, "flexflow_amd", "libflexflow_c.so")
    if not os.path.exists(lib):
        sys.path.insert(0, ROOT)
        import build_ext
        build_ext.build_capi()
    exe = str(tmp_path / "mlp_c")
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "csrc", "capi"), os.path.join(ROOT, "tests", "capi", "mlp_c.c"),
                    "-L", os.path.dirname(lib), "-lflexflow_c", f"-Wl,-rpath,{os.path.dirname(lib)}", "-lm", "-o", exe],
                   check=True)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "loss" in r.stdout
