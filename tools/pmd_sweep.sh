#!/bin/bash
# Poll-mode kernel sweeps: tile size (COP_PPT) at the driver's 20-batch
# post, with tile/phase stamps (tools/pmd_probe.py) and the 20-step bench
# line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-pmd_sweep}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 120 "$out/probe_ppt4_phases.log" env COP_PMD_STAMPS=2 python3 -u "$R/tools/pmd_probe.py" --posts 1,20 --iters 20
step 120 "$out/probe_ppt1.log" env COP_PPT=1 python3 -u "$R/tools/pmd_probe.py" --posts 1,20 --iters 20
step 120 "$out/probe_ppt1_phases.log" env COP_PPT=1 COP_PMD_STAMPS=2 python3 -u "$R/tools/pmd_probe.py" --posts 1,20 --iters 20
step 120 "$out/probe_ppt8.log" env COP_PPT=8 python3 -u "$R/tools/pmd_probe.py" --posts 1,20 --iters 20
step 200 "$out/bench20_ppt1.log" env COP_PPT=1 python3 -u "$R/bench.py" --no-cpu --steps 20 --warmup 5
step 200 "$out/bench20_ppt4.log" python3 -u "$R/bench.py" --no-cpu --steps 20 --warmup 5
