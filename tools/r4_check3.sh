#!/bin/bash
# GPU tests (all, up to 5 failures), the multi-ring drop-in diagnosis,
# carry on/off A/B of the poll-mode kernel, then the route-form A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check3
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 500 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "PASSED|FAILED|ERROR" "$out/pytest.log" | grep -v PASSED | head -20
step 120 "$out/rings_diag_3_seq.log" python3 -u "$R/tools/rings_diag.py" 3 0
step 120 "$out/rings_diag_3_thr.log" python3 -u "$R/tools/rings_diag.py" 3 1
step 120 "$out/rings_diag_1_seq.log" python3 -u "$R/tools/rings_diag.py" 1 0
cd "$R" && step 400 "$out/ab_carry.log" bash tools/ab_pmd.sh "$out/carry" "carry:" "nocarry:COP_PMD_CARRY=0" "carry2:" "nocarry2:COP_PMD_CARRY=0"
cat "$out/ab_carry.log" | tail -4
bash "$R/tools/r4_bkt.sh"
echo done
