#!/bin/bash
# PMC calibration runs with known byte / probe counts (tools/membench,
# tools/probebench), left under gpurun_out/calib/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/calib
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pmc_fetch_mb.log" rocprofv3 --pmc FETCH_SIZE -d "$out/fetch_mb" -o mb --output-format csv -- "$R/tools/membench"
step 300 "$out/pmc_write_mb.log" rocprofv3 --pmc WRITE_SIZE -d "$out/write_mb" -o mb --output-format csv -- "$R/tools/membench"
step 300 "$out/pmc_dram_mb.log" rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d "$out/dram_mb" -o mb --output-format csv -- "$R/tools/membench"
step 300 "$out/pmc_req_pb.log" rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -d "$out/req_pb" -o pb --output-format csv -- "$R/tools/probebench"
step 300 "$out/pmc_dram_pb.log" rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d "$out/dram_pb" -o pb --output-format csv -- "$R/tools/probebench"
step 300 "$out/pmc_fetch_pb.log" rocprofv3 --pmc FETCH_SIZE -d "$out/fetch_pb" -o pb --output-format csv -- "$R/tools/probebench"
