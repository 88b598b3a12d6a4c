#!/bin/bash
# instrumented builds of the product library (phase cycle counters, per-env block times), for tools/phase_prof.py and
# tools/timeline.py: the default 16-lane GJK build and the Golf tasks' 8-lane one (URGYM_LIB selects)
set -e
cd "$(dirname "$0")/.."
F="-O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -shared -std=c++17 -Wno-unused-value -Wno-unused-result -DUG_PROF"
/opt/rocm/bin/hipcc $F -o urgym_amd/_lib/liburgym_prof.so urgym_amd/csrc/ug_capi.hip
/opt/rocm/bin/hipcc $F -DUG_GJK_G=8 -o urgym_amd/_lib/liburgym_prof_g8.so urgym_amd/csrc/ug_capi.hip
