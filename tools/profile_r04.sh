#!/bin/bash
# Round-4 measurements, left under gpurun_out/r04/ (copied into profiles/r04/):
#   bench20       the driver's command (fw1k, 20 steps, poll-mode kernel)
#   c5_bench20    config 5 at 20 steps (the poll-mode stall check: 5 runs)
#   dense20       the driver's command with dense lists (what the drop-in consumes)
#   pmd_pmc       PMC traffic of the poll-mode kernel over exactly K posted
#                 batches (tools/pmc_pmd.py) + the membench calibration passes
#   ring          the drop-in ring loop: 1 loop sync / async / pmd, 5 loops sync / pmd
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --steps 20 --warmup 5
step 200 "$out/c5_bench20.log" python3 -u "$R/bench.py" --quick --workload fw_lpm_1m --steps 20 --warmup 5
step 200 "$out/dense20.log" python3 -u "$R/bench.py" --quick --lists dense --steps 20 --warmup 5
step 200 "$out/pmd_pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/pmd_fetch" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
step 200 "$out/pmd_pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/pmd_write" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
step 200 "$out/mb_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/mb_fetch" -o mb --output-format csv -- "$R/tools/membench"
step 200 "$out/mb_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/mb_write" -o mb --output-format csv -- "$R/tools/membench"
for m in sync async pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $a
done
for m in sync pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $a
done
echo done
