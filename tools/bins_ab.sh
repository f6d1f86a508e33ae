#!/bin/bash
# Per-rule hit counters by binning vs one atomic per hit: parity tests, then
# A/B on config 5 (1M rules + 1M prefixes) and on fw1k with counters, the
# config-5 bench line, and its rocprof stats + PMC traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-bins_ab}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/pytest_rules.log" python3 -u -m pytest "$R/tests/test_gpu_rules.py" "$R/tests/test_gpu_tables.py" -x -v --timeout 300 --timeout-method thread
step 400 "$out/fw_lpm_1m_L25_ctr.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 --rule-counters \
    bins atomics:COP_HIT_BINS=0
step 240 "$out/fw1k_L384_ctr.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 384 --rounds 5 --launches 4 --rule-counters \
    bins atomics:COP_HIT_BINS=0
step 400 "$out/bench_fw_lpm_1m.log" python3 -u "$R/bench.py" --workload fw_lpm_1m --no-cpu --steps 768 --warmup 384
"$R/tools/profile_round.sh" "${1:-bins_ab}_c5" --workload fw_lpm_1m --steps 768 --warmup 384
