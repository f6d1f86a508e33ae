#!/bin/bash
# rocprofv3 kernel stats (csv) of the driver's command; poll-mode steady
# state with records and lists staged in LDS (whole-line output) against
# the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/final2
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/stats20.log" rocprofv3 --kernel-trace --stats -d "$out/stats20" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu
cd "$R" && step 500 "$out/ab.log" bash tools/ab_pmd.sh "$out/ab" "cur:" "stage:COP_PMD_REC=stage COP_STAGE_LISTS=1" "cur2:" "stage2:COP_PMD_REC=stage COP_STAGE_LISTS=1"
tail -4 "$out/ab.log"
echo done
