#!/bin/bash
# poll-mode tests with the restructured carry; bucketed route form v3
# (64-byte pair read) against DIR-24-8; carry on/off A/B (x3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check7
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -8
B="$R/bench.py --workload fw_lpm --steps 1024 --warmup 256 --no-cpu --secondary none"
for f in dir bkt dir bkt; do
  step 200 "$out/fw_lpm_${f}.log" python3 -u $B --route-form $f
  grep -h '^{"metric"' "$out/fw_lpm_${f}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], d["value"], "frac", r["frac"], "kernel_ms", r["kernel_ms_per_launch"])' "$f"
done
cd "$R" && step 400 "$out/ab_cur.log" bash tools/ab_pmd.sh "$out/cur" "cur:" "cur2:"
cat "$out/ab_cur.log" | tail -2
echo done
