#!/bin/bash
# held last-step stores: poll-mode tests, then hold on/off A/B (x3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check10
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pytest.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" "$R/tests/test_gpu_seg.py" "$R/tests/test_gpu_rings.py" "$R/tests/test_gpu_dropin.py" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -4
cd "$R" && step 600 "$out/ab.log" bash tools/ab_pmd.sh "$out/ab" "hold:" "nohold:COP_PMD_HOLD=0" "hold2:" "nohold2:COP_PMD_HOLD=0" "hold3:" "nohold3:COP_PMD_HOLD=0"
tail -6 "$out/ab.log"
echo done
