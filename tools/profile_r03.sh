#!/bin/bash
# Round-3 profiles of one workload (segmented lists, the bench's defaults),
# left under gpurun_out/p3_<workload>/ (copied into profiles/r03/ afterwards):
#   stats  rocprofv3 --kernel-trace --stats of the driver's command (20 steps,
#          poll-mode kernel) plus the bench's one-shot roofline launches
#   fetch / write / dram: --pmc FETCH_SIZE, --pmc WRITE_SIZE and
#          --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum (separate passes) of
#          one-shot launches (--engine launch), the kernel the roofline quotes
# usage: tools/profile_r03.sh <workload> [extra bench args]
set -o pipefail
wl=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/p3_$wl
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
B="$R/bench.py --quick --workload $wl"
step 400 "$out/stats.log" rocprofv3 --kernel-trace --stats -d "$out/stats" -o bench --output-format csv -- python3 $B --steps 20 --warmup 5 "$@"
L="--engine launch --steps 2048 --warmup 0 --repeats 1"
step 400 "$out/pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o bench --output-format csv -- python3 $B $L "$@"
step 400 "$out/pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o bench --output-format csv -- python3 $B $L "$@"
step 400 "$out/pmc_dram.log" rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d "$out/dram" -o bench --output-format csv -- python3 $B $L "$@"
