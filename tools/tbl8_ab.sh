#!/bin/bash
# Packed tbl8 groups: table parity tests, then A/B against plain groups on
# FW + LPM 100k and on config 5 (1M rules + 1M prefixes), with and without
# per-rule counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-tbl8_ab}
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pytest_tables.log" python3 -u -m pytest "$R/tests/test_gpu_tables.py" "$R/tests/test_gpu_rules.py" -x -v --timeout 200 --timeout-method thread
step 240 "$out/fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 \
    plain:COP_TBL8=plain packed:COP_TBL8=packed
step 400 "$out/fw_lpm_1m_L25_ctr.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 --rule-counters \
    plain:COP_TBL8=plain packed:COP_TBL8=packed
step 400 "$out/fw_lpm_1m_L25.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 \
    plain:COP_TBL8=plain packed:COP_TBL8=packed
