set -o pipefail
mkdir -p gpurun_out/r4diag
B="python3 -u bench.py --quick --workload fw_lpm_1m --steps 20 --warmup 5"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4diag/pytest.log 2>&1 && \
COP_PMD_PREWARM=0 COP_COLL_PREWARM=0 timeout -k 10 150 $B > gpurun_out/r4diag/v1_none.log 2>&1 && \
COP_PMD_PREWARM=1 COP_COLL_PREWARM=0 timeout -k 10 150 $B > gpurun_out/r4diag/v3_pmdonly.log 2>&1 && \
timeout -k 10 150 $B > gpurun_out/r4diag/v2_both.log 2>&1 && \
for m in "" async; do COP_HOST_PROF=1 timeout -k 10 60 tools/ringbench 8388608 16384 1 $m >> gpurun_out/r4diag/ring.log 2>&1 || exit 7; done
rc=$?; tail -3 gpurun_out/r4diag/pytest.log; grep -h "timed\|rccl\|ms_per" gpurun_out/r4diag/v*.log | cut -c1-300; cat gpurun_out/r4diag/ring.log; exit $rc
