#!/bin/bash
# the side-kernel probe over the cases that tell resources from queues apart
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/side
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
export COP_PMD_IDLE_MS=3000
step 60 "$out/a_100k.log" python3 -u "$R/tools/pmd_side_probe.py" 100000
step 60 "$out/b_100k_percu3.log" env COP_PMD_PER_CU=3 python3 -u "$R/tools/pmd_side_probe.py" 100000
step 60 "$out/c_100k_hwq8.log" env GPU_MAX_HW_QUEUES=8 python3 -u "$R/tools/pmd_side_probe.py" 100000
step 60 "$out/d_100k_nobins.log" env COP_HIT_BINS=0 python3 -u "$R/tools/pmd_side_probe.py" 100000
step 60 "$out/e_fw1k.log" python3 -u "$R/tools/pmd_side_probe.py" 1000
step 60 "$out/f_100k_noprewarm.log" env COP_PMD_PREWARM=0 python3 -u "$R/tools/pmd_side_probe.py" 100000
grep -h "^{" $out/*.log
