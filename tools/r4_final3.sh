#!/bin/bash
# Round-4 final check of the final code (after the staged forward lists):
# the driver's tiers, rocprofv3 stats of the driver's command, the poll-mode
# PMC over exactly 1024 batches (+ membench calibration), config 5 at 20
# steps, the ring loops
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/final3
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 600 "$out/pytest_gpu.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread
grep -E "FAILED|ERROR|passed|failed" "$out/pytest_gpu.log" | tail -4
step 300 "$out/smoke.log" python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 300 "$out/bench20.log" python3 -u "$R/bench.py" --gpus 1 --steps 20 --warmup 5
step 500 "$out/bench_default.log" python3 -u "$R/bench.py"
step 300 "$out/stats20.log" rocprofv3 --kernel-trace --stats -d "$out/stats20" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu
step 200 "$out/pmd_pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/pmd_fetch" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
step 200 "$out/pmd_pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/pmd_write" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
step 200 "$out/mb_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/mb_fetch" -o mb --output-format csv -- "$R/tools/membench"
step 200 "$out/mb_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/mb_write" -o mb --output-format csv -- "$R/tools/membench"
step 200 "$out/c5_bench20.log" python3 -u "$R/bench.py" --quick --workload fw_lpm_1m --steps 20 --warmup 5
for m in sync async pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $a
  COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $a
done
grep -h "aggregate" $out/ring*.log
grep -h '^{"metric"' "$out/bench20.log" "$out/bench_default.log" | cut -c1-300
echo done
