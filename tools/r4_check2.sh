#!/bin/bash
# GPU tests, config 5 at 20 steps, the ring loops (pinned), and the
# next-tile L2 prefetch experiment against the production kernel (poll-mode
# steady state: bench without --quick)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/check2
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 120 --timeout-method thread
step 200 "$out/c5_bench20.log" python3 -u "$R/bench.py" --quick --workload fw_lpm_1m --steps 20 --warmup 5
for m in sync async pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $a
done
for m in sync async pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $a
done
grep -h "Mpkt/s aggregate" $out/ring*.log
cd "$R" && step 400 "$out/ab_pf.log" bash tools/ab_pmd.sh "$out/pf" "cur:" "pf:COP_LIB=$R/ghost-dataplane_amd/libcopgpu_pf.so COP_PMD_PREFETCH=1" "cur2:" "pf2:COP_LIB=$R/ghost-dataplane_amd/libcopgpu_pf.so COP_PMD_PREFETCH=1"
cat "$out/ab_pf.log"
echo done
