#!/bin/bash
# tools/sanitize.sh -- ASan + UBSan run of the host-side code on the CPU (SURVEY §5 "race
# detection / sanitizers"): liba5x.so with its host half instrumented (table parser and
# $HEX / -t merge, word split, partition, hit / plain formatting, the C-ABI argument
# checks; the gfx950 device code is untouched: every -fsanitize sits after -Xarch_host)
# and the C oracle, both under clang's shared sanitizer runtime, then the CPU test suite
# through them.  GPU AddressSanitizer is not available on the GPU pool; this is CPU only.
#
#   bash tools/sanitize.sh [pytest args]      -> log in gpurun_out/sanitize.log
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R" || exit 2
LLVM=/opt/rocm/lib/llvm
RT=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
OUT=$R/hashcat_a5_table_generator_amd/_build_asan
OOUT=$R/oracle/_build_asan
mkdir -p "$OUT" "$OOUT" gpurun_out
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
-Xarch_host -fno-omit-frame-pointer -Xarch_host -shared-libsan"
C=$R/hashcat_a5_table_generator_amd/csrc
if [ ! -f "$OUT/liba5x.so" ] || [ -n "$(find $C include -newer $OUT/liba5x.so -type f | head -1)" ]; then
  echo "building $OUT/liba5x.so (host ASan + UBSan)"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -fvisibility=hidden $SAN \
    -I include -I $C $C/a5x_kernels.hip $C/a5x_modes.hip $C/a5x_digest.hip $C/a5x_host.cpp \
    -o $OUT/liba5x.so || exit 3
fi
echo "building $OOUT/liba5oracle.so (ASan + UBSan)"
$LLVM/bin/clang -O1 -g -std=c11 -fPIC -shared -pthread -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -fno-omit-frame-pointer -shared-libsan oracle/a5_oracle.c -o $OOUT/liba5oracle.so || exit 4
# python is not instrumented: the runtime is preloaded; leaks of the interpreter are not ours
export LD_PRELOAD=$RT
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export A5X_LIB_PATH=$OUT/liba5x.so A5X_ORACLE_LIB=$OOUT/liba5oracle.so A5X_SANITIZED=1
python -m pytest tests/ -q -m "not gpu" -p no:cacheprovider "$@" 2>&1 | tee gpurun_out/sanitize.log
rc=$?
grep -E "ERROR: AddressSanitizer|runtime error:" gpurun_out/sanitize.log && rc=5
echo "sanitize rc=$rc"
exit $rc
