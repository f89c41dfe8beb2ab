#!/bin/bash
# The CPU test suite against the host-sanitised library (build.py --asan): AddressSanitizer + UBSan on the host
# entry points (gp_pcg64_seed_state, the table builders, gp_argmax_multinomial_distribution, gp_zig_log1p_neg,
# gp_exp_libm, gp_create's config checks ...). Python itself is not instrumented, so the clang ASan runtime is
# preloaded; leak checking is off (the interpreter's own allocations would dominate it).
set -eo pipefail
cd "$(dirname "$0")/.."
python gym-po-taxi_amd/build.py --asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export GYM_PO_AMD_LIB=$PWD/gym-po-taxi_amd/gym_po_amd/libgympo_amd_asan.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD=$RT python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
