#!/bin/bash
# ISA inspection of one poll-mode kernel instantiation (no GPU needed):
# FW = interval form, no route stage, coalesced slots, PPT = $1 (1 or 4),
# extra defines in $KDEFS. Prints VGPR/SGPR/scratch and writes the
# disassembly to /tmp/isa/pmd_probe.s.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
ppt=${1:-1}
mkdir -p /tmp/isa
cd /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$R/include" -I"$R/ghost-dataplane_amd/csrc" \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -DCOPK_FW_PART=1 -DCOPK_ISA_PROBE=$ppt $KDEFS \
  -c "$R/ghost-dataplane_amd/csrc/cop_pmd.hip" -o probe.o
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=probe.fat probe.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=probe.fat --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=probe.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes probe.co | grep -E "\.name:|vgpr_count|sgpr_count|private_segment_fixed" | grep -B3 -A0 "" | paste - - - - | grep "Lb0" | awk '{print $2, $4, $6, $8}'
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn probe.co > pmd_probe.s
