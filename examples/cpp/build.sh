#!/bin/bash
# Build every C++ example against the C API (libflexflow_c.so; build it first with
# `python -c "import build_ext; build_ext.build_capi()"`). Binaries land next to their sources.
#   examples/cpp/build.sh [example-dir ...]
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
LIB="$ROOT/flexflow_amd"
CXX="${CXX:-g++}"
dirs=("$@")
[ ${#dirs[@]} -eq 0 ] && dirs=(AlexNet ResNet resnext50 InceptionV3 MLP_Unify DLRM XDL candle_uno Transformer
                               mixture_of_experts split_test split_test_2)
for d in "${dirs[@]}"; do
  for src in "$HERE/$d"/*.cc; do
    out="${src%.cc}"
    "$CXX" -std=c++17 -O2 -Wall -I"$ROOT/csrc/capi" -I"$HERE" "$src" -L"$LIB" -lflexflow_c \
      -Wl,-rpath,"$LIB" -o "$out"
  done
done
