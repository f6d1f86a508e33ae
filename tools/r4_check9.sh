#!/bin/bash
# poll-mode store visibility: write-through stores (production) against
# plain stores + one agent release per tile (libcopgpu_rel.so), and plain
# stores with no release (libcopgpu_nowt.so, timing only); the poll-mode
# tests on the release build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check9
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
L=$R/ghost-dataplane_amd
COP_LIB=$L/libcopgpu_rel.so step 300 "$out/pytest_rel.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" "$R/tests/test_gpu_seg.py" "$R/tests/test_gpu_rings.py" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest_rel.log" | tail -4
cd "$R" && step 600 "$out/ab.log" bash tools/ab_pmd.sh "$out/ab" "wt:" "rel:COP_LIB=$L/libcopgpu_rel.so" "nowt:COP_LIB=$L/libcopgpu_nowt.so" "wt2:" "rel2:COP_LIB=$L/libcopgpu_rel.so" "nowt2:COP_LIB=$L/libcopgpu_nowt.so"
tail -6 "$out/ab.log"
echo done
