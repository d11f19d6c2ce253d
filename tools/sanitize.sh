#!/usr/bin/env bash
# Host-only AddressSanitizer + UndefinedBehaviorSanitizer build and run of the native code
# (SURVEY.md §5.2).  -fsanitize is applied to the HOST compilation only (-Xarch_host);
# GPU code objects are unaffected and never run here.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/mxdesk-sanitize"
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
SRC=("$ROOT/tools/sanitize_main.cpp" "$ROOT/csrc/codec/h264_encoder.cpp" "$ROOT/csrc/codec/h264_cpu.cpp"
     "$ROOT/csrc/codec/h264_kernels.hip" "$ROOT/csrc/codec/h264_deblock.hip" "$ROOT/csrc/codec/hevc_cpu.cpp" "$ROOT/csrc/codec/hevc_encoder.cpp"
     "$ROOT/csrc/codec/hevc_kernels.hip" "$ROOT/csrc/codec/vp8_bitstream.cpp" "$ROOT/csrc/codec/vp8_cpu.cpp"
     "$ROOT/csrc/codec/vp8_gpu.cpp" "$ROOT/csrc/codec/vp8_kernels.hip" "$ROOT/csrc/net/srtp.cpp" "$ROOT/csrc/net/dtls.cpp"
     "$ROOT/csrc/net/rtp_h264.cpp" "$ROOT/csrc/net/rtp_h265.cpp" "$ROOT/csrc/net/rtp_vp8.cpp" "$ROOT/csrc/net/sctp.cpp" "$ROOT/csrc/net/rtp_sender.cpp")
objs=()
for s in "${SRC[@]}"; do
  o="$OUT/$(basename "$s").o"
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -std=c++17 -O1 -g $SAN -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN "${objs[@]}" -o "$OUT/sanitize" -lssl -lcrypto
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/sanitize"
