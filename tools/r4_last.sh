#!/bin/bash
# last check of the committed tree: GPU tests, smoke, the driver's command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/last
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 600 "$out/pytest_gpu.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest_gpu.log" | tail -4
step 300 "$out/smoke.log" python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5
grep -h '^{"metric"' "$out/bench20.log" | cut -c1-300
echo done
