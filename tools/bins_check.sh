#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/bins3
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/pytest_rules.log" python3 -u -m pytest "$R/tests/test_gpu_rules.py" "$R/tests/test_gpu_tables.py" -x -v --timeout 300 --timeout-method thread
step 400 "$out/fw_lpm_1m_L25_ctr.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 --rule-counters bins atomics:COP_HIT_BINS=0
step 240 "$out/fw1k_L384_ctr.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 384 --rounds 5 --launches 4 --rule-counters bins atomics:COP_HIT_BINS=0
step 400 "$out/bench_fw_lpm_1m.log" python3 -u "$R/bench.py" --workload fw_lpm_1m --no-cpu --steps 768 --warmup 384
step 120 "$out/gather_probe.log" "$R/tools/gather_probe" 1048576
