#!/bin/bash
# What the driver runs at round end, on one box: the GPU test suite,
# smoke(), the driver's bench command and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-round_check}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 900 "$out/pytest_gpu.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread
step 300 "$out/smoke.log" python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5
step 400 "$out/bench_default.log" python3 -u "$R/bench.py"
