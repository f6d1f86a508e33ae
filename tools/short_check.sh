#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/short2
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 200 "$out/short_probe.log" python3 -u "$R/tools/short_probe.py" --ppts 0,4,8 --lens 1,4,20
step 200 "$out/short_probe_ppt1.log" python3 -u "$R/tools/short_probe.py" --ppts 1 --lens 1,4
step 200 "$out/stamps_short.log" python3 -u "$R/tools/stamps.py" short
