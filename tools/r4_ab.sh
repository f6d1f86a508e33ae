#!/bin/bash
# round-4 check: GPU tests, config 5 at 20 steps (poll-mode pause around the
# side work), A/B of the driver's command (this build / round 3's / no gate),
# the drop-in ring loop with pinned threads
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/ab
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 120 --timeout-method thread
step 200 "$out/c5_bench20.log" python3 -u "$R/bench.py" --quick --workload fw_lpm_1m --steps 20 --warmup 5
for i in 1 2; do
  for v in cur r3 nogate; do
    lib=""; [ $v = r3 ] && lib=$R/ghost-dataplane_amd/libcopgpu_r3.so; [ $v = nogate ] && lib=$R/ghost-dataplane_amd/libcopgpu_nogate.so
    COP_LIB=$lib step 200 "$out/ab_${v}_$i.log" python3 -u "$R/bench.py" --quick --steps 20 --warmup 5 --repeats 21
    python3 "$R/tools/summ.py" "$out/ab_${v}_$i.log" | head -1
  done
done
for m in sync async pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $a
done
for m in sync pmd; do
  a=""; [ $m != sync ] && a=$m
  COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $a
done
grep -h "Mpkt/s aggregate\|prof loop0" $out/ring*.log
echo done
