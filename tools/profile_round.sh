#!/bin/bash
# Profile the bench's default configuration on the GPU box and leave the
# summaries under gpurun_out/prof_<tag>/ (copied into profiles/ afterwards):
#   1. rocprofv3 --kernel-trace --stats of the full bench command
#   2. rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of a
#      shorter bench run and of tools/membench (calibration: known bytes)
#   3. tools/pmc_traffic.py -> per-launch HBM traffic JSON
# usage: tools/profile_round.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 400 "$out/stats.log" rocprofv3 --kernel-trace --stats -d "$out/stats" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu "$@"
step 400 "$out/pmc_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 3072 --warmup 3072 "$@"
step 400 "$out/pmc_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 3072 --warmup 3072 "$@"
step 300 "$out/pmc_fetch_mb.log" rocprofv3 --pmc FETCH_SIZE -d "$out/fetch_mb" -o mb --output-format csv -- "$R/tools/membench"
step 300 "$out/pmc_write_mb.log" rocprofv3 --pmc WRITE_SIZE -d "$out/write_mb" -o mb --output-format csv -- "$R/tools/membench"
python3 "$R/tools/pmc_traffic.py" "$out/fetch/bench_counter_collection.csv" "$out/write/bench_counter_collection.csv" \
    "$out/fetch_mb/mb_counter_collection.csv" "$out/write_mb/mb_counter_collection.csv" "$out/traffic.json"
