#!/usr/bin/env bash
# Build tools/diag/pack4_repro.hip, record the compiler version and the packing ISA of each
# kernel under $OUT (default profiles/r03_pack4), and run it when a GPU is present.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${OUT:-$ROOT/profiles/r03_pack4}"
mkdir -p "$OUT"
/opt/rocm/bin/hipcc --version > "$OUT/compiler_version.txt" 2>&1
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 --cuda-device-only -S "$ROOT/tools/diag/pack4_repro.hip" -o "$OUT/pack4_repro_gfx950.s"
for k in k_shift_or k_perm k_masked k_site_recon; do
  awk -v k="$k" '$0 ~ "^_Z[0-9]+"k"PKiPji:" {p=1} p {print} p && /s_endpgm/ {exit}' "$OUT/pack4_repro_gfx950.s" > "$OUT/isa_$k.s"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 "$ROOT/tools/diag/pack4_repro.hip" -o "${TMPDIR:-/tmp}/pack4_repro"
if [ -e /dev/kfd ]; then "${TMPDIR:-/tmp}/pack4_repro" | tee "$OUT/run.txt"; fi
