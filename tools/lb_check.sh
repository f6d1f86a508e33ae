#!/bin/bash
# Look-back / small-launch check: GPU suite, short launches (1/4/20
# batches, tickets vs blockIdx order), phase stamps, the 1024-batch kernel
# A/B and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-lb_check}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 900 "$out/pytest_gpu.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 300 --timeout-method thread
step 200 "$out/short_probe.log" python3 -u "$R/tools/short_probe.py" --ppts 0 --lens 1,4,20
step 200 "$out/short_probe_tickets.log" env COP_STATIC_ORDER=0 python3 -u "$R/tools/short_probe.py" --ppts 0 --lens 1,4,20
step 200 "$out/stamps_short.log" python3 -u "$R/tools/stamps.py" short
step 240 "$out/ab_fw1k_L1024.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 1024 --rounds 5 --launches 4 base
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu
