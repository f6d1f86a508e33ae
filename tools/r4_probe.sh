#!/bin/bash
# where a 20-batch post spends its time now (phase stamps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/probe
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 200 "$out/probe.log" python3 -u "$R/tools/pmd_probe.py" --posts 1,20,128 --iters 30
COP_PMD_STAGE_LIST=0 step 200 "$out/probe_env.log" python3 -u "$R/tools/pmd_probe.py" --posts 20 --iters 30
echo done
