#!/bin/bash
# instrumented build of the product library (phase cycle counters), for tools/phase_prof.py
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -shared -std=c++17 \
  -Wno-unused-value -Wno-unused-result -DUG_PROF -o urgym_amd/_lib/liburgym_prof.so urgym_amd/csrc/ug_capi.hip
