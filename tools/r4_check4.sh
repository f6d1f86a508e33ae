#!/bin/bash
# multi-ring drop-in: diagnosis with and without the per-tile system acquire,
# then the poll-mode / ring / drop-in GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check4
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 120 "$out/rings_diag_3_seq.log" python3 -u "$R/tools/rings_diag.py" 3 0
COP_PMD_ACQUIRE=0 step 120 "$out/rings_diag_3_seq_noacq.log" python3 -u "$R/tools/rings_diag.py" 3 0
step 120 "$out/rings_diag_3_thr.log" python3 -u "$R/tools/rings_diag.py" 3 1
step 120 "$out/rings_diag_1_seq.log" python3 -u "$R/tools/rings_diag.py" 1 0
step 300 "$out/pytest.log" python3 -u -m pytest "$R/tests/test_gpu_dropin.py" "$R/tests/test_gpu_pmd.py" "$R/tests/test_gpu_rings.py" "$R/tests/test_gpu_seg.py" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -8
for m in pmd; do
  COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $m
  COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $m
done
grep -h "aggregate" $out/ring*.log
echo done
