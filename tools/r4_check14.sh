#!/bin/bash
# DIR-24-8 stages on the poll-mode step-by-step path (probes one step
# ahead): GPU tests, then FW + LPM at 20 steps stepwise on/off, fw1k driver
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check14
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 500 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -4
for v in steps tb steps tb; do
  e=""; [ $v = tb ] && e="COP_PMD_STEPWISE=0"
  env $e "$R/tools/gpu_step.sh" 200 "$out/fw_lpm20_$v.log" python3 -u "$R/bench.py" --workload fw_lpm --steps 20 --warmup 5 --no-cpu --secondary none --repeats 11 || exit 99
  grep -h '^{"metric"' "$out/fw_lpm20_$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; p=d.get("pmd",{}); print(sys.argv[1], d["value"], "timed", r.get("frac_timed"), "steady", p.get("steady_frac"))' "$v"
done
cd "$R" && step 300 "$out/ab.log" bash tools/ab_pmd.sh "$out/ab" "cur:" "cur2:"
tail -2 "$out/ab.log"
echo done
