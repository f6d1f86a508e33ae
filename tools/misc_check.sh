#!/bin/bash
# The driver's bench command (poll-mode fields), and tile size on config 5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-misc}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu
step 400 "$out/c5_ppt.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 --rule-counters \
    base p4:COP_PPT=4 p1:COP_PPT=1
