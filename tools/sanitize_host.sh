#!/usr/bin/env bash
# Host ASan + UBSan run (SURVEY.md 5 "race detection / sanitizers"): builds the sanitizer variant of
# libfhe_rocm.so (`make -C fhe-sign_amd asan`, -fsanitize on the host compilation only) and runs the
# CPU tests that exercise the host code paths with untrusted or intricate memory handling --
# the validating deserializers (corrupted / truncated / oversized inputs), key generation and
# encryption, the BIP-340 signer, the level scheduler and progress marks, and the host-fold / dry
# engine runs of the BigUintFHE mul (the compat carry-count chain) and the simulated runs of every radix
# algorithm (Karatsuba, division, shifts, the column form) -- against it.  CPU only: no GPU, and
# GPU-side sanitizers are not available on the GPU pool.
# Usage: tools/sanitize_host.sh [log]   (default log: profiles/r5/sanitize_host_r5.log)
set -euo pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r5/sanitize_host_r5.log}
mkdir -p "$(dirname "$LOG")"
make -C fhe-sign_amd asan -j8 >/dev/null
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(find /opt/rocm/lib/llvm -name 'libclang_rt.asan-x86_64.so' | head -1)
{
  echo "# host sanitizer run: $(date -u +%FT%TZ), $(git rev-parse --short HEAD 2>/dev/null || echo nogit)"
  echo "# runtime: $RT"
  echo "# flags: -fsanitize=address,undefined -fno-sanitize-recover=undefined (host code only)"
  # leak detection off: the Python interpreter itself does not free everything at exit
  echo "# instrumented: $(nm -D fhe-sign_amd/lib_asan/libfhe_rocm.so | grep -c '__asan_report\|__ubsan_handle') sanitizer hooks referenced"
  LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0 FHE_ROCM_LIB="$PWD/fhe-sign_amd/lib_asan/libfhe_rocm.so" \
    python -c "import sys; sys.path.insert(0, 'fhe-sign_amd'); from fhe_sign import _lib; _lib.load(); print('# loaded', _lib.LIB_PATH)"
  st=0
  LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  FHE_ROCM_LIB="$PWD/fhe-sign_amd/lib_asan/libfhe_rocm.so" \
    python -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_serialize.py tests/test_keys.py \
      tests/test_schnorr.py tests/test_scheduler.py tests/test_abi.py tests/test_biguint_host.py \
      tests/test_radix_sim.py 2>&1 || st=$?
  echo "# exit status: $st"
} | tee "$LOG"
grep -q "ERROR: AddressSanitizer\|runtime error:" "$LOG" && { echo "sanitizer findings, see $LOG"; exit 1; }
grep -q "# exit status: 0" "$LOG"
