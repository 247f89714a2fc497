"""C++ examples (examples/cpp/*, reference examples/cpp/*): every model written against the C++ API
(csrc/capi/flexflow.hpp over libflexflow_c.so) compiles, and trains for one step in --small mode.
On CPU here (the embedded runtime's CPU path); tests/test_cpp_examples_gpu.py runs them on cuda:0."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "cpp")
PROGRAMS = ["AlexNet/alexnet", "ResNet/resnet", "resnext50/resnext", "InceptionV3/inception", "MLP_Unify/mlp",
            "DLRM/dlrm", "XDL/xdl", "candle_uno/candle_uno", "Transformer/transformer", "mixture_of_experts/moe",
            "split_test/split_test", "split_test_2/split_test_2"]

# the examples are rebuilt when their source or any API header is newer than the binary
_HDRS = max(os.path.getmtime(os.path.join(ROOT, "csrc", "capi", h)) for h in ("flexflow_c.h", "flexflow.hpp"))


def build_examples():
    if not os.path.exists(os.path.join(ROOT, "flexflow_amd", "libflexflow_c.so")):
        sys.path.insert(0, ROOT)
        import build_ext
        build_ext.build_capi()
    missing = [p for p in PROGRAMS if not os.path.exists(os.path.join(EX, p))
               or os.path.getmtime(os.path.join(EX, p)) < max(os.path.getmtime(os.path.join(EX, p + ".cc")), _HDRS)]
    if missing:
        subprocess.run([os.path.join(EX, "build.sh")] + sorted({p.split("/")[0] for p in missing}), check=True)


def run_examples(progs, extra_env, extra_args=(), parallel=4, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), **extra_env)
    out = {}
    for i in range(0, len(progs), parallel):
        procs = {p: subprocess.Popen([os.path.join(EX, p), "-b", "4", "--iterations", "2", "--small", *extra_args],
                                     env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for p in progs[i:i + parallel]}
        for p, pr in procs.items():
            try:
                txt, _ = pr.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                pr.kill()
                txt, _ = pr.communicate()
            out[p] = (pr.returncode, txt)
    return out


def check(results):
    for p, (rc, txt) in results.items():
        assert rc == 0, f"{p} exited {rc}:\n{txt[-3000:]}"
        last = [ln for ln in txt.splitlines() if "THROUGHPUT" in ln]
        assert last, f"{p}: no throughput line\n{txt[-2000:]}"
        loss = float(last[-1].split("loss")[1].split(",")[0])
        assert loss == loss and loss < 1e4, f"{p}: loss {loss}"


def test_cpp_examples_train_on_cpu():
    build_examples()
    check(run_examples(PROGRAMS, {"CUDA_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "2"}))


def test_cpp_api_multi_output_layers():
    """split / top_k / group_by through the C++ API return the right number of tensors (moe and
    split_test_2 use them); the composite ff.moe path agrees in shape with the explicit one."""
    build_examples()
    check(run_examples(["mixture_of_experts/moe"], {"CUDA_VISIBLE_DEVICES": ""}, ("--composite",)))
