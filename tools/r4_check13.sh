#!/bin/bash
# step-by-step tiles with the list staged in LDS (16-byte stores): tests,
# then A/B against word stores (libcopgpu_c0.so) and the LDS-staged
# tile_body form (COP_PMD_REC=stage)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check13
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
L=$R/ghost-dataplane_amd
step 300 "$out/pytest.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" "$R/tests/test_gpu_seg.py" "$R/tests/test_gpu_rings.py" "$R/tests/test_gpu_dropin.py" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -4
cd "$R" && step 700 "$out/ab.log" bash tools/ab_pmd.sh "$out/ab" "c16:" "c0:COP_LIB=$L/libcopgpu_c0.so" "c16b:" "c0b:COP_LIB=$L/libcopgpu_c0.so"
tail -6 "$out/ab.log"
echo done
