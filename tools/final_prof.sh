#!/bin/bash
# Round-end profiles with the final code: the driver's bench command (fw1k)
# and config 5, each with rocprofv3 --kernel-trace --stats and the
# FETCH_SIZE / WRITE_SIZE passes (after one plain run of the driver's
# command).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/${1:-final}"
"$R/tools/gpu_step.sh" 300 "$R/gpurun_out/${1:-final}/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5 || exit 99
"$R/tools/profile_round.sh" "${1:-final}_fw1k" --steps 20 --warmup 5 || exit 99
"$R/tools/profile_round.sh" "${1:-final}_c5" --workload fw_lpm_1m --steps 768 --warmup 384 || exit 99
