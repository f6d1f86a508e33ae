#!/bin/bash
# The A/B tables DESIGN.md quotes, re-measured with the current kernel
# (interleaved rounds in one process per workload; tools/ab.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/ab_r02
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 240 "$out/fw1k_L1024.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 1024 --rounds 5 --launches 4 \
    base strided:COP_LOADS=strided p4:COP_PPT=4 lists_from_regs:COP_STAGE_LISTS=0 nocompact/nocompact \
    static_tiles:COP_DBG=2 no_lds_staging:COP_DBG=4 no_counter_atomics:COP_DBG=1 no_lookback_wait:COP_DBG=32 \
    lds_pad20k:COP_LDS_PAD=20480 lds_pad40k:COP_LDS_PAD=40960
step 240 "$out/fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 \
    base strided:COP_LOADS=strided p4:COP_PPT=4 nocompact/nocompact
step 240 "$out/imix_L384.log" python3 -u "$R/tools/ab.py" --workload imix --per-launch 384 --rounds 5 --launches 4 \
    base p1:COP_PPT=1 p8:COP_PPT=8
for L in 96 384 1024; do
    step 240 "$out/fw1k_per_launch_$L.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch $L --rounds 5 --launches 8 base
done
