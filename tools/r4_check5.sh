#!/bin/bash
# GPU tests; bucketed route form (two-pair scan) against DIR-24-8 at tile
# sizes 2048 / 1024; poll-mode steady state under tile size, workers per CU
# and carry
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check5
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 500 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --maxfail=8 --timeout 120 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -8
B="$R/bench.py --workload fw_lpm --steps 1024 --warmup 256 --no-cpu --secondary none"
for v in dir:0 bkt:0 bkt:4 dir:4 bkt:0; do
  f=${v%%:*}; ppt=${v#*:}
  if [ "$ppt" = 0 ]; then unset COP_PPT; else export COP_PPT=$ppt; fi
  step 200 "$out/fw_lpm_${f}_ppt${ppt}.log" python3 -u $B --route-form $f
  unset COP_PPT
  grep -h '^{"metric"' "$out/fw_lpm_${f}_ppt${ppt}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], d["value"], "frac", r["frac"], "kernel_ms", r["kernel_ms_per_launch"])' "$v"
done
cd "$R" && step 600 "$out/ab_steady.log" bash tools/ab_pmd.sh "$out/steady" "cur:" "ppt8:COP_PPT=8" "percu4:COP_PMD_PER_CU=4" "nocarry:COP_PMD_CARRY=0" "cur2:" "ppt8b:COP_PPT=8"
cat "$out/ab_steady.log" | tail -6
echo done
