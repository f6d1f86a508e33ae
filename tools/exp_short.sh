#!/bin/bash
# Short-run (20-step) experiments: bench variants and the poll-mode probe.
# usage: tools/exp_short.sh <outdir-name> [variant...]   variants: base nocompact cu4 probe probe2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-exp_short}; shift
mkdir -p "$out"
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
for v in "$@"; do
  case $v in
    base) step 200 "$out/bench20_base.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    nocompact) step 200 "$out/bench20_nocompact.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 --no-compact ;;
    cu4) COP_PMD_PER_CU=4 step 200 "$out/bench20_cu4.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    probe) COP_PMD_STAMPS=1 step 200 "$out/probe.log" python3 -u "$R/tools/pmd_probe.py" --posts 1,20 ;;
    probe2) COP_PMD_STAMPS=2 step 200 "$out/probe2.log" python3 -u "$R/tools/pmd_probe.py" --posts 1,20 ;;
    recstage) COP_PMD_REC=stage step 200 "$out/bench20_recstage.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    pmdtests) step 300 "$out/pytest_pmd.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" -m gpu -x -v --timeout 120 --timeout-method thread ;;
    gputests) step 600 "$out/pytest_gpu.log" python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread ;;
    nodefer) COP_PMD_DEFER_CTR=0 step 200 "$out/bench20_nodefer.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    tabletests) step 300 "$out/pytest_tables.log" python3 -u -m pytest "$R/tests/test_gpu_tables.py" -m gpu -x -v --timeout 120 --timeout-method thread ;;
    abtrie) step 300 "$out/ab_trie_fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 dir trie:COP_LPM_FORM=trie ;;
    abtrie_imix) step 300 "$out/ab_trie_imix_L384.log" python3 -u "$R/tools/ab.py" --workload imix --per-launch 384 --rounds 5 --launches 4 dir trie:COP_LPM_FORM=trie ;;
    abtrie_1m) step 300 "$out/ab_trie_fw_lpm_1m_L25.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 dir trie:COP_LPM_FORM=trie ;;
    ppt1) COP_PPT=1 step 200 "$out/bench20_ppt1.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 5 ;;

    ppt4) COP_PPT=4 step 200 "$out/bench20_ppt4.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 5 ;;
    ppt8) COP_PPT=8 step 200 "$out/bench20_ppt8.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 5 ;;
    relay16) COP_PMD_RELAY_STRIDE=16 step 200 "$out/bench20_relay16.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    relay256) COP_PMD_RELAY_STRIDE=256 step 200 "$out/bench20_relay256.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 ;;
    abrec) step 300 "$out/ab_rec_fw1k_L1024.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 1024 --rounds 7 --launches 4 base paired:COP_REC_PAIRED=1 base2 paired2:COP_REC_PAIRED=1 &&
           step 300 "$out/ab_rec_fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 base paired:COP_REC_PAIRED=1 ;;
    pairedtests) COP_REC_PAIRED=1 step 600 "$out/pytest_paired.log" python3 -u -m pytest "$R/tests/test_gpu_parity.py" "$R/tests/test_gpu_ring.py" "$R/tests/test_gpu_golden.py" "$R/tests/test_gpu_demux.py" -m gpu -x -q --timeout 300 --timeout-method thread ;;
    abbase) step 300 "$out/ab_fw1k_L1024.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 1024 --rounds 7 --launches 4 base &&
            step 300 "$out/ab_fw1k_L96.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 96 --rounds 7 --launches 8 base &&
            step 300 "$out/ab_fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 base &&
            step 300 "$out/ab_imix_L384.log" python3 -u "$R/tools/ab.py" --workload imix --per-launch 384 --rounds 5 --launches 4 base ;;
    stamps) step 200 "$out/stamps_short.log" python3 -u "$R/tools/stamps.py" short ;;
    abnt) step 300 "$out/ab_nt_fw_lpm_L1024.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 5 --launches 4 base nt:COP_PROBE_NT=1 &&
          step 300 "$out/ab_nt_fw_lpm_1m_L25.log" python3 -u "$R/tools/ab.py" --workload fw_lpm_1m --per-launch 25 --rounds 5 --launches 8 base nt:COP_PROBE_NT=1 &&
          step 300 "$out/ab_nt_imix_L384.log" python3 -u "$R/tools/ab.py" --workload imix --per-launch 384 --rounds 5 --launches 4 base nt:COP_PROBE_NT=1 ;;
    abstream) for rep in 1 2; do for L in base w2 w4 w2e6; do
                 if [ $L = base ]; then lib=libcopgpu.so; else lib=libcopgpu_$L.so; fi
                 COP_LIB=$R/ghost-dataplane_amd/$lib step 200 "$out/ab_stream_${L}_fw1k_$rep.log" python3 -u "$R/tools/ab.py" --workload fw1k --per-launch 1024 --rounds 3 --launches 4 $L || exit 99
               done; done
               for L in base w2 w4 w2e6; do
                 if [ $L = base ]; then lib=libcopgpu.so; else lib=libcopgpu_$L.so; fi
                 COP_LIB=$R/ghost-dataplane_amd/$lib step 200 "$out/ab_stream_${L}_fw_lpm.log" python3 -u "$R/tools/ab.py" --workload fw_lpm --per-launch 1024 --rounds 3 --launches 4 $L || exit 99
               done ;;
    fwlpm) step 300 "$out/bench_fw_lpm.log" python3 -u "$R/bench.py" --workload fw_lpm --steps 20 --warmup 5 --no-cpu --repeats 5 ;;
    pf) COP_PMD_PREFETCH=1 step 200 "$out/bench20_pf.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 5 ;;
    pfdefault) COP_PMD_PREFETCH=1 step 300 "$out/bench_default_pf.log" python3 -u "$R/bench.py" --engine pmd --no-cpu --repeats 3 &&
               step 300 "$out/bench_default_pmd.log" python3 -u "$R/bench.py" --engine pmd --no-cpu --repeats 3 ;;
    pftests) COP_PMD_PREFETCH=1 step 300 "$out/pytest_pmd_pf.log" python3 -u -m pytest "$R/tests/test_gpu_pmd.py" -m gpu -x -v --timeout 120 --timeout-method thread ;;
    relayN) for st in 128 512 1280 256; do COP_PMD_RELAY_STRIDE=$st step 200 "$out/bench20_relay$st.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 || exit 99; done ;;
    launch) step 200 "$out/bench20_launch.log" python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu --repeats 21 --engine launch ;;
  esac
done
