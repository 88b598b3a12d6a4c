#!/bin/bash
# The CPU restatement under AddressSanitizer + UBSan (host code only; fatal on the first report): builds
# oracle/_build/libugoracle_asan.so (make -C oracle asan) and runs the oracle's CPU tests against it -- the golden
# vectors of every task, the known-answer tests, the GJK / EPA restatement, and tests/test_oracle_crafted.py's crafted
# states (capacity overflows in both contact modes, the 480 cap, the split pass, the non-finite guard).  Python loads
# the instrumented library through ctypes, so the sanitizer runtimes are preloaded into the interpreter.
# Usage: bash tools/oracle_asan.sh [pytest args]   (log: profiles/round4_oracle_asan.txt when run with --record)
set -eu
cd "$(dirname "$0")/.."
make -s -C oracle asan
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
RECORD=0
if [ "${1:-}" = "--record" ]; then RECORD=1; shift; fi
TESTS="tests/test_oracle_crafted.py tests/test_oracle_kat.py tests/test_gjk.py tests/test_golden.py tests/test_golden_box.py
       tests/test_golden_cubes.py tests/test_golden_golf.py tests/test_golden_twoballs.py tests/test_golden_variants.py
       tests/test_box_kat.py tests/test_dynamics_kat.py"
run() {
    LD_PRELOAD="$ASAN:$UBSAN" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
        UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 URGYM_ORACLE_LIB="$PWD/oracle/_build/libugoracle_asan.so" \
        python -m pytest $TESTS -q -m "not gpu" -p no:cacheprovider "$@"
}
if [ $RECORD = 1 ]; then
    { echo "# tools/oracle_asan.sh ($(date -u +%F)): oracle/_build/libugoracle_asan.so, $(gcc --version | head -1)"; run "$@"; } \
        > profiles/round4_oracle_asan.txt 2>&1
    tail -3 profiles/round4_oracle_asan.txt
else
    run "$@"
fi
