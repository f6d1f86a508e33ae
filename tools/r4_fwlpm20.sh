#!/bin/bash
# FW + LPM 100k at the driver's 20 steps (poll-mode kernel), route form
# DIR-24-8 against the bucketed L2 form, two runs each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/fwlpm20
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
for f in dir bkt dir bkt; do
  step 200 "$out/fw_lpm20_$f.log" python3 -u "$R/bench.py" --workload fw_lpm --steps 20 --warmup 5 --no-cpu --secondary none --route-form $f --repeats 11
  grep -h '^{"metric"' "$out/fw_lpm20_$f.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; p=d.get("pmd",{}); print(sys.argv[1], d["value"], "timed", r.get("frac_timed"), "steady", p.get("steady_frac"), "frac", r["frac"])' "$f"
done
echo done
