#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer build of the CPU side (the
# host library libwtfhost: core + modules, the oracle liboracle.so, the twin,
# hostcheck, and the host build of the engine's lane code tests/native/
# sim_lane.cc) into build/asan/, then the CPU test suite against it
# (tests/cpu_bins.py: WTF_CPU_BUILD). Any sanitizer report fails the run.
#   scripts/sanitize_cpu.sh [pytest args]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/asan
mkdir -p "$OUT/obj"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1"
CXX="g++ -std=c++20 -fPIC -fopenmp $SAN"
CC="gcc -std=gnu99 -fPIC $SAN"
H=$ROOT/wtf_amd/host
cd "$H"
SRCS="wtf_api.cc kdmp.cc blake3_lite.cc host_pool.cc module_slots.cc module_instances.cc runner.cc mutator_lite.cc net_exchange.cc
      wire.cc remote.cc merge_block.cc modules/fuzzer_tlv_server.cc modules/crash_detection_umode.cc modules/fuzzer_hevd.cc"
objs=()
pids=()
for s in $SRCS; do
  o=$OUT/obj/$(echo "$s" | tr / _).o
  objs+=("$o")
  $CXX -c -o "$o" "$s" & pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
for p in "${pids[@]}"; do wait "$p"; done
rm -f "$OUT/libwtfhost.a" && ar rcs "$OUT/libwtfhost.a" "${objs[@]}"
cd "$ROOT/oracle"
$CC -shared -o "$OUT/liboracle.so" x86_oracle.c
$CC -c -o "$OUT/obj/x86_oracle.o" x86_oracle.c
$CXX -rdynamic -o "$OUT/wtf_twin" twin_backend.cc "$OUT/obj/x86_oracle.o" -Wl,--whole-archive "$OUT/libwtfhost.a" -Wl,--no-whole-archive
$CXX -DWTF_AMD_HOST -o "$OUT/hostcheck" hostcheck.cc -Wl,--whole-archive "$OUT/libwtfhost.a" -Wl,--no-whole-archive
cd "$ROOT/tests/native"
g++ -std=c++17 -DWTFGPU_HOST_SIM -fPIC -shared $SAN -o "$OUT/libsimlane.so" sim_lane.cc
echo "built $OUT"
cd "$ROOT"
# the Python process loads sanitized shared objects: the runtimes go first
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export WTF_CPU_BUILD=$OUT
python -m pytest -q -m "not gpu" -p no:cacheprovider "$@" tests/
