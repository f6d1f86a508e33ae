#!/bin/bash
# One GPU lease: named steps, in order, each under its own time limit
# (tools/gpu_step.sh: a fault-like exit ends the call there).
#
# usage (through gpurun, from the repo root):
#   bash tools/lease.sh <out> <step> [<step> ...]
# <out>: directory under gpurun_out/ for the logs (e.g. r05/check1).
# Steps:
#   pytest          every -m gpu test (one process)
#   pytest:<expr>   the -m gpu tests matching -k <expr>
#   smoke           __graft_entry__.smoke()
#   bench20         the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench_default   bench.py with no flags
#   slots           the driver's command at --slots static / reuse / always (quick, 11 runs each)
#   stats20         rocprofv3 --kernel-trace --stats of the driver's command
#   pmc_pmd         FETCH_SIZE / WRITE_SIZE passes over a 1024-batch poll-mode post + membench calibration
#   c5              config 5 (fw_lpm_1m) at 20 steps, quick, route form $C5_FORM (dir)
#   c5_forms        config 5 in every FW x route form: dir/dir, dir/bkt, bkt/bkt (quick)
#   imix            FW + LPM 100k IMIX at 20 steps (quick)
#   rings           the ring loops (tools/ringbench: 1 and 5 loops, sync / async / pmd)
#   probe           tools/pmd_probe.py stamps of the 20-batch post
# Extra arguments for bench steps: $BENCH_ARGS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
line() { grep -h '^{"metric"' "$@" | cut -c1-400; }
B="python3 -u $R/bench.py"
for s in "$@"; do
  case $s in
    pytest)
      step 900 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 120 --timeout-method thread
      grep -E "FAILED|ERROR|passed|failed" "$out/pytest.log" | tail -6 ;;
    pytest:*)
      k=${s#pytest:}
      step 600 "$out/pytest_${k//[^A-Za-z0-9_]/_}.log" python3 -u -m pytest "$R/tests" -m gpu -v -k "$k" --timeout 120 --timeout-method thread
      grep -E "FAILED|ERROR|passed|failed" "$out/pytest_${k//[^A-Za-z0-9_]/_}.log" | tail -6 ;;
    smoke)
      step 300 "$out/smoke.log" python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench20)
      step 600 "$out/bench20.log" $B --gpus 1 --steps 20 --warmup 5 $BENCH_ARGS
      line "$out/bench20.log" ;;
    bench_default)
      step 600 "$out/bench_default.log" $B $BENCH_ARGS
      line "$out/bench_default.log" ;;
    slots)
      for v in static reuse always static reuse always; do
        step 200 "$out/slots_$v.log" $B --quick --steps 20 --warmup 5 --repeats 11 --slots $v $BENCH_ARGS
        echo "$v $(line "$out/slots_$v.log" | cut -c1-200)"
      done ;;
    stats20)
      step 300 "$out/stats20.log" rocprofv3 --kernel-trace --stats -d "$out/stats20" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu $BENCH_ARGS ;;
    pmc_pmd)
      step 200 "$out/pmd_pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/pmd_fetch" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
      step 200 "$out/pmd_pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/pmd_write" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --batches 1024
      step 200 "$out/mb_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/mb_fetch" -o mb --output-format csv -- "$R/tools/membench"
      step 200 "$out/mb_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/mb_write" -o mb --output-format csv -- "$R/tools/membench" ;;
    pmc_all)
      # every workload of the line, both engines: poll-mode FETCH_SIZE /
      # WRITE_SIZE over one lifetime serving exactly K posted batches
      # (tools/pmc_pmd.py), one-shot passes over bench.py --quick of that
      # workload alone; membench calibration once (reduce on the CPU with
      # tools/pmc_pmd.py reduce and tools/pmc_traffic.py)
      for wk in ${PMC_WORKLOADS:-fw1k:1024 fw_lpm:1024 fw_lpm_imix:384 fw_lpm_1m:384}; do
        w=${wk%%:*}; k=${wk##*:}
        step 300 "$out/pmd_${w}_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/pmd_${w}_fetch" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --workload "$w" --batches "$k"
        step 300 "$out/pmd_${w}_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/pmd_${w}_write" -o pmd --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --workload "$w" --batches "$k"
        step 400 "$out/os_${w}_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/os_${w}_fetch" -o os --output-format csv -- python3 "$R/bench.py" --quick --workload "$w" --steps 20 --warmup 5 --secondary none --no-cpu
        step 400 "$out/os_${w}_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/os_${w}_write" -o os --output-format csv -- python3 "$R/bench.py" --quick --workload "$w" --steps 20 --warmup 5 --secondary none --no-cpu
      done
      step 200 "$out/mb_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/mb_fetch" -o mb --output-format csv -- "$R/tools/membench"
      step 200 "$out/mb_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/mb_write" -o mb --output-format csv -- "$R/tools/membench" ;;
    pmc_l2)
      # L2 hits and misses of the poll-mode kernel over exactly K posted
      # batches, per workload (the probes' L2 miss ratio beside the traffic)
      for wk in ${PMC_WORKLOADS:-fw1k:1024 fw_lpm:1024}; do
        w=${wk%%:*}; k=${wk##*:}
        step 300 "$out/l2_${w}.log" rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/l2_${w}" -o l2 --output-format csv -- python3 "$R/tools/pmc_pmd.py" run --workload "$w" --batches "$k"
      done ;;
    pmc_oneshot)
      # the one-shot kernel's PMC passes over the driver's command (reduce
      # here with tools/pmc_traffic.py and the membench passes of pmc_pmd)
      step 300 "$out/os_pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/os_fetch" -o os --output-format csv -- python3 "$R/bench.py" --quick --steps 20 --warmup 5 --secondary none --no-cpu
      step 300 "$out/os_pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/os_write" -o os --output-format csv -- python3 "$R/bench.py" --quick --steps 20 --warmup 5 --secondary none --no-cpu ;;
    n2)
      # two ranks sharing the one GPU (one-shot launches: two persistent
      # kernels cannot both hold every CU), through the start gate; config
      # 5's RCCL init fails on a shared GPU and every rank skips the reduce
      step 600 "$out/n2_shared.log" $B --gpus 2 --allow-shared-gpu --engine launch --steps 20 --warmup 5 --no-cpu --no-rccl-check --secondary fw_lpm_1m
      grep -h '^{"metric"' "$out/n2_shared.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("n2", d["value"], "overlap", d["windows_overlap"], "union", d["value_union"], "skew", d["windows"]["start_skew_us_median"], "c5", {k: d["secondary"]["fw_lpm_1m"].get(k) for k in ("value", "windows_overlap", "rccl_init", "error")})' ;;
    win1)
      # a one-step load window (libcopgpu_win1.so, -DCOPK_PMD_WIN=1) against
      # the then-default two-step window, alternating, then both tails
      # (profiles/r05/check8; one step has been the default since)
      i=0
      for lib in main win1 main win1 main win1; do
        i=$((i + 1))
        L=""; [ "$lib" = win1 ] && L="$R/ghost-dataplane_amd/libcopgpu_win1.so"
        COP_LIB=$L step 300 "$out/win_${lib}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/win_${lib}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("win", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "dyn steady", p.get("dynamic_tiles", {}).get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$lib"
      done
      step 300 "$out/tail_main.log" python3 -u "$R/tools/pmd_tail.py" --posts 60
      COP_LIB="$R/ghost-dataplane_amd/libcopgpu_win1.so" step 300 "$out/tail_win1.log" python3 -u "$R/tools/pmd_tail.py" --posts 60
      grep -h "post->done\|slot on CU (w // 256)  [04]" "$out/tail_main.log" "$out/tail_win1.log" ;;
    ab:*)
      # an experiment build (ghost-dataplane_amd/libcopgpu_<name>.so) against
      # the default build on the driver's command, alternating three pairs,
      # then both tails of the 20-batch post (tools/pmd_tail.py)
      x=${s#ab:}; i=0
      for lib in main $x main $x main $x; do
        i=$((i + 1))
        L=""; [ "$lib" != main ] && L="$R/ghost-dataplane_amd/libcopgpu_$x.so"
        COP_LIB=$L step 300 "$out/ab_${lib}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/ab_${lib}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("ab", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "dyn steady", p.get("dynamic_tiles", {}).get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"), "16 in flight", p.get("one_batch_posts", {}).get("mpkt_s"))' "$lib"
      done
      step 300 "$out/tail_main.log" python3 -u "$R/tools/pmd_tail.py" --posts 60
      COP_LIB="$R/ghost-dataplane_amd/libcopgpu_$x.so" step 300 "$out/tail_$x.log" python3 -u "$R/tools/pmd_tail.py" --posts 60
      grep -h "post->done\|slot on CU (w // 256)  [04]" "$out/tail_main.log" "$out/tail_$x.log" ;;
    abx:*)
      # an experiment build against the default build on the workload of
      # $BENCH_ARGS (e.g. --workload fw_lpm_imix), alternating three pairs:
      # the poll-mode 20-step value and the one-shot kernel's frac (no tails)
      x=${s#abx:}; i=0
      for lib in main $x main $x main $x; do
        i=$((i + 1))
        L=""; [ "$lib" != main ] && L="$R/ghost-dataplane_amd/libcopgpu_$x.so"
        COP_LIB=$L step 300 "$out/abx_${lib}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/abx_${lib}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); r=d["roofline"]; rl=d.get("roofline_launch", r); print("abx", sys.argv[1], d["value"], "timed", r["frac_timed"], "probe", r.get("probe_bound"), "launch frac", rl["frac"], "launch probe", rl.get("probe_bound"), "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$lib"
      done ;;
    envab:*)
      # an environment setting (envab:NAME=VALUE) against the default on the
      # driver's command, alternating three pairs, then the poll-mode,
      # segmented and ring GPU tests with it set
      kv=${s#envab:}; i=0
      for v in off on off on off on; do
        i=$((i + 1))
        if [ $v = on ]; then
          env "$kv" "$R/tools/gpu_step.sh" 300 "$out/env_${v}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS || exit 99
        else
          step 300 "$out/env_${v}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        fi
        grep -h '^{"metric"' "$out/env_${v}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("env", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "dyn steady", p.get("dynamic_tiles", {}).get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$v"
      done
      env "$kv" "$R/tools/gpu_step.sh" 600 "$out/pytest_env.log" python3 -u -m pytest "$R/tests" -m gpu -v -k "pmd or seg or rings or rewritten" --timeout 120 --timeout-method thread || exit 99
      grep -E "FAILED|ERROR|passed|failed" "$out/pytest_env.log" | tail -4 ;;
    steps_ab)
      # the poll-mode FW + LPM 100k post with step-by-step tiles (the route's
      # DIR-24-8 probes pipelined across steps) against whole-tile bodies
      # ($COP_PMD_STEPWISE=0), alternating, at the driver's 20 steps
      i=0
      for v in 0 1 0 1 0 1; do
        i=$((i + 1))
        COP_PMD_STEPWISE=$v step 300 "$out/steps_fwlpm_${v}_$i.log" $B --workload fw_lpm --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/steps_fwlpm_${v}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("stepwise", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$v"
      done ;;
    e2e)
      # the end-to-end host-memory path (mbuf pool -> pinned staging -> H2D ->
      # pipeline -> D2H), 1..16 gather threads, first pass checked bit-exact
      step 300 "$out/e2e.log" python3 -u "$R/tools/e2e.py"
      tail -8 "$out/e2e.log" ;;
    c5)
      step 300 "$out/c5_${C5_FORM:-dir}.log" $B --quick --workload fw_lpm_1m --steps 20 --warmup 5 --route-form "${C5_FORM:-dir}" $BENCH_ARGS
      line "$out/c5_${C5_FORM:-dir}.log" ;;
    c5_forms)
      for f in "dir dir" "dir bkt" "bkt bkt" "bkt dir"; do
        set -- $f
        step 300 "$out/c5_fw$1_rt$2.log" $B --quick --workload fw_lpm_1m --steps 20 --warmup 5 --fw-form "$1" --route-form "$2" $BENCH_ARGS
        grep -h '^{"metric"' "$out/c5_fw$1_rt$2.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("fw", sys.argv[1], "route", sys.argv[2], d["value"], "kernel frac", r["frac"], "ms/launch", r["kernel_ms_per_launch"], "timed", r["frac_timed"])' "$1" "$2"
      done ;;
    imix)
      step 300 "$out/imix20.log" $B --quick --workload fw_lpm_imix --steps 20 --warmup 5 $BENCH_ARGS
      line "$out/imix20.log" ;;
    rings)
      for m in sync async pmd; do
        a=""; [ $m != sync ] && a=$m
        COP_HOST_PROF=1 step 90 "$out/ring1_$m.log" "$R/tools/ringbench" 8388608 16384 1 $a
        COP_HOST_PROF=1 step 120 "$out/ring5_$m.log" "$R/tools/ringbench" 8388608 16384 5 $a
      done
      grep -h "aggregate" "$out"/ring*.log ;;
    dyn)
      # dynamic tiles ($COP_PMD_DYN=1) against the static order, alternating
      i=0
      for v in 0 1 0 1; do
        i=$((i + 1))
        COP_PMD_DYN=$v step 300 "$out/dyn${v}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/dyn${v}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("dyn", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$v"
      done ;;
    acq)
      # slot-reuse modes at the driver's 20 steps ($COP_PMD_ACQUIRE: 0 none,
      # 1 acquire every tile, 3 coherent loads every tile), then the
      # rewritten-slot tests with coherent loads every tile / once wrapped
      for v in 0 1 3 4 0 1 3 4; do
        COP_PMD_ACQUIRE=$v step 200 "$out/acq$v.log" $B --quick --steps 20 --warmup 5 --repeats 11 $BENCH_ARGS
        echo "acq=$v $(grep -h '^\[rank 0\] fw1k: timed' "$out/acq$v.log" | cut -c1-120)"
      done
      for v in 3 4; do
        COP_PMD_ACQUIRE=$v step 300 "$out/pytest_acq$v.log" python3 -u -m pytest "$R/tests" -m gpu -v -k "rewritten or rings or pmd_seg" --timeout 120 --timeout-method thread
        grep -E "FAILED|ERROR|passed|failed" "$out/pytest_acq$v.log" | tail -4
      done ;;
    reuse)
      # the default slot-reuse guard against declared-static slots, with the
      # poll-mode steady state (1024-batch posts wrap the 1024-slot pool)
      for v in static reuse static reuse; do
        step 300 "$out/reuse_$v.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check --slots $v $BENCH_ARGS
        grep -h '^{"metric"' "$out/reuse_$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("slots", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$v"
      done ;;
    outmem)
      # outputs in uncached / fine-grained HBM with plain (not write-through)
      # stores (libcopgpu_wt0.so: -DCOPK_PMD_WT=0) against HBM + write-through
      for v in device:main uncached:wt0 fine:wt0 device:main uncached:wt0; do
        mem=${v%%:*}; lib=${v##*:}
        L=""; [ "$lib" = wt0 ] && L="$R/ghost-dataplane_amd/libcopgpu_wt0.so"
        COP_LIB=$L step 300 "$out/outmem_$mem.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check --out-mem $mem $BENCH_ARGS
        grep -h '^{"metric"' "$out/outmem_$mem.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("out", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"))' "$v"
      done ;;
    tail)
      step 300 "$out/tail.log" python3 -u "$R/tools/pmd_tail.py" --posts 60 --dump "$out/tail.npz"
      cat "$out/tail.log" ;;
    rings_ab)
      # the poll-mode drop-in loops: coherent loads on every tile (3, the
      # default for host rings) against an acquire on every tile (1)
      for v in 3 1 3 1; do
        COP_PMD_ACQUIRE=$v step 120 "$out/ring5_pmd_acq$v.log" "$R/tools/ringbench" 8388608 16384 5 pmd
        COP_PMD_ACQUIRE=$v step 90 "$out/ring1_pmd_acq$v.log" "$R/tools/ringbench" 8388608 16384 1 pmd
        echo "acq=$v $(grep -h aggregate "$out/ring5_pmd_acq$v.log") / $(grep -h aggregate "$out/ring1_pmd_acq$v.log")"
      done ;;
    dyn4)
      # dynamic 1024-packet tiles with a two-step window (libcopgpu_win2.so,
      # -DCOPK_PMD_WIN=2, $COP_PMD_DYN=4) against the static order in the
      # same build and in the default build
      i=0
      for v in main:0 win2:0 win2:4 main:0 win2:0 win2:4; do
        i=$((i + 1)); lib=${v%%:*}; d=${v##*:}
        L=""; [ "$lib" = win2 ] && L="$R/ghost-dataplane_amd/libcopgpu_win2.so"
        COP_LIB=$L COP_PMD_DYN=$d step 300 "$out/dyn4_${lib}_${d}_$i.log" $B --steps 20 --warmup 5 --repeats 11 --secondary none --no-cpu --no-rccl-check $BENCH_ARGS
        grep -h '^{"metric"' "$out/dyn4_${lib}_${d}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("pmd",{}); print("dyn4", sys.argv[1], d["value"], "timed", d["roofline"]["frac_timed"], "steady", p.get("steady_frac"), "one-batch", p.get("single_batch_post_to_done_us_median"), p.get("workers"))' "$v"
      done
      COP_LIB="$R/ghost-dataplane_amd/libcopgpu_win2.so" COP_PMD_DYN=4 step 600 "$out/pytest_dyn4.log" python3 -u -m pytest "$R/tests" -m gpu -v -k "pmd or seg or rings" --timeout 120 --timeout-method thread
      grep -E "FAILED|ERROR|passed|failed" "$out/pytest_dyn4.log" | tail -4 ;;
    pytest_dyn)
      COP_PMD_DYN=1 step 600 "$out/pytest_dyn.log" python3 -u -m pytest "$R/tests" -m gpu -v -k "pmd or seg or rings or dropin" --timeout 120 --timeout-method thread
      grep -E "FAILED|ERROR|passed|failed" "$out/pytest_dyn.log" | tail -6 ;;
    probe)
      step 200 "$out/probe.log" python3 -u "$R/tools/pmd_probe.py" ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
