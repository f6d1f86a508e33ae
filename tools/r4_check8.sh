#!/bin/bash
# bucketed route form at 5 waves per SIMD against DIR-24-8 (x2), its tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check8
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread -k "bkt or fw_lpm_100k or imix_fw_lpm or tables"
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -4
B="$R/bench.py --workload fw_lpm --steps 1024 --warmup 256 --no-cpu --secondary none"
for f in dir bkt dir bkt; do
  step 200 "$out/fw_lpm_${f}.log" python3 -u $B --route-form $f
  grep -h '^{"metric"' "$out/fw_lpm_${f}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], d["value"], "frac", r["frac"], "kernel_ms", r["kernel_ms_per_launch"])' "$f"
done
for f in dir bkt; do
  step 200 "$out/imix_${f}.log" python3 -u $R/bench.py --workload fw_lpm_imix --steps 1024 --warmup 256 --no-cpu --secondary none --route-form $f
  grep -h '^{"metric"' "$out/imix_${f}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("imix", sys.argv[1], d["value"], "frac", r["frac"], "kernel_ms", r["kernel_ms_per_launch"])' "$f"
done
cd "$R" && step 500 "$out/ab_wt.log" bash tools/ab_pmd.sh "$out/wt" "wt:" "nowt:COP_LIB=$R/ghost-dataplane_amd/libcopgpu_nowt.so" "wt2:" "nowt2:COP_LIB=$R/ghost-dataplane_amd/libcopgpu_nowt.so"
tail -4 "$out/ab_wt.log"
echo done
