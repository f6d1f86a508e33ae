#!/bin/bash
# Poll-mode kernel check after a change: its GPU tests, the post timeline
# (tools/pmd_probe.py), the driver's 20-step bench line and the default
# bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-pmd_check}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pytest_pmd.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" -x -v --timeout 120 --timeout-method thread
step 120 "$out/probe.log" python3 -u "$R/tools/pmd_probe.py" --posts 1,20,64 --iters 20
step 120 "$out/probe_phases.log" env COP_PMD_STAMPS=2 python3 -u "$R/tools/pmd_probe.py" --posts 1,20,64 --iters 20
step 200 "$out/bench20.log" python3 -u "$R/bench.py" --no-cpu --steps 20 --warmup 5
step 300 "$out/bench_default.log" python3 -u "$R/bench.py" --no-cpu
