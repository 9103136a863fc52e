#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code:
# the oracle (C) and the C-ABI host layer of libjwave_hip.so (capi.cpp:
# validation, pass planner, staging) rebuilt with -fsanitize=address,undefined
# (hipcc: host side only, -Xarch_host), then the CPU test suite runs against
# those builds.  GPU code is not sanitized (not available on this pool).
# usage: tools/sanitize.sh            (CPU only; writes build/asan/)
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd); cd $R
O=$R/build/asan; mkdir -p $O
CLANG=/opt/rocm/lib/llvm/bin/clang
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
$CLANG $SAN -shared-libsan -fPIC -ffp-contract=off -std=c11 -shared \
  oracle/jwave_oracle.c oracle/jwave_oracle_par.c -lm -lpthread -o $O/libjwave_oracle.so
C=jwave_amd/csrc
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -x hip \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer \
  -c $C/capi.cpp -o $O/capi.o
OBJS=$(ls build/obj/*.o | grep -v capi.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -shared-libsan -fsanitize=address,undefined \
  -o $O/libjwave_hip.so $OBJS $O/capi.o
RT=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)
echo "runtime: $RT"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
JWAVE_AMD_LIB=$O/libjwave_hip.so JWAVE_ORACLE_LIB=$O/libjwave_oracle.so \
  python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
# proof of what ran: the sanitized builds are the ones mapped into the process
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0 JWAVE_AMD_LIB=$O/libjwave_hip.so \
JWAVE_ORACLE_LIB=$O/libjwave_oracle.so python - <<'PY'
import sys
sys.path[:0] = [".", "oracle"]
import jwave_amd._lib as L, oracle
L.lib(); oracle.lib()
print("mapped:", sorted({l.split()[-1] for l in open("/proc/self/maps")
                         if "libjwave" in l or "asan" in l}))
PY
