#!/bin/bash
# Host sanitizer pass: the CPU-only sources built with gcc's AddressSanitizer +
# UndefinedBehaviorSanitizer (eds-bwt_amd: format.cpp, index_io.cpp, eds_transform, the CLI,
# edsbwt_gen, stringCheck -> _build_asan/; the oracle -> oracle/_build_asan/), then the whole CPU
# test suite (`-m "not gpu"`) against them: the Python process preloads libasan + libubsan, the
# tools run as sanitized executables.  Any ASan report or UBSan finding aborts the test that hit it.
#   bash tools/asan_suite.sh [pytest args...]     (log: stdout)
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -j 8 -C eds-bwt_amd asan
make -s -C oracle asan
export EDSBWT_LIB=$PWD/eds-bwt_amd/_build_asan/libedsbwt.so
export EDSBWT_BUILD_DIR=$PWD/eds-bwt_amd/_build_asan
export EDSBWT_ORACLE_BUILD=$PWD/oracle/_build_asan
# reports go to files as well (pytest captures the test's stderr): $ASAN_LOG_DIR/asan.<pid>, ubsan.<pid>
ASAN_LOG_DIR=${ASAN_LOG_DIR:-$PWD/.wt/asan_logs}
rm -rf "$ASAN_LOG_DIR"; mkdir -p "$ASAN_LOG_DIR"
export ASAN_OPTIONS=detect_leaks=0:detect_odr_violation=0:halt_on_error=1:abort_on_error=1:log_path=$ASAN_LOG_DIR/asan
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$ASAN_LOG_DIR/ubsan
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
echo "[asan] EDSBWT_LIB=$EDSBWT_LIB EDSBWT_ORACLE_BUILD=$EDSBWT_ORACLE_BUILD LD_PRELOAD=$LD_PRELOAD"
nm -D "$EDSBWT_LIB" | grep -c " U __asan_" | sed 's/^/[asan] libedsbwt.so ASan-instrumented references: /'
nm -D oracle/_build_asan/liboracle.so | grep -c " U __asan_" | sed 's/^/[asan] liboracle.so ASan-instrumented references: /'
rc=0
python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" || rc=$?
for f in "$ASAN_LOG_DIR"/*; do [ -f "$f" ] && { echo "== $f"; cat "$f"; }; done
echo "[asan] sanitizer reports: $(ls "$ASAN_LOG_DIR" | wc -l); pytest exit $rc"
exit $rc
