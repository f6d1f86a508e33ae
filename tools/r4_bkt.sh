#!/bin/bash
# Route-form A/B on FW + LPM 100k (BASELINE configs[3]; and the IMIX
# config[2]): DIR-24-8 / bucketed intervals (COP_BKT_XBITS 0..2) / trie,
# one-shot launches, plus PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss)
# of the dir and bkt kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r04/bkt
mkdir -p "$out"
export TMPDIR=/tmp
step() { "$R/tools/gpu_step.sh" "$@" || exit 99; }
step 300 "$out/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -x -v --timeout 120 --timeout-method thread -k "bkt or fw_lpm_100k or imix_fw_lpm"
B="$R/bench.py --workload fw_lpm --steps 1024 --warmup 256 --no-cpu --secondary none"
for v in dir bkt:1 bkt:0 bkt:2 trie; do
  f=${v%%:*}; x=${v#*:}; [ "$x" = "$v" ] && x=1
  COP_BKT_XBITS=$x step 200 "$out/fw_lpm_${f}${x}.log" python3 -u $B --route-form $f
  grep -h '^{"metric"' "$out/fw_lpm_${f}${x}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], d["value"], "frac", r["frac"], "frac_timed", r.get("frac_timed"), "probes", json.dumps(r.get("table_probes")))' "$v"
done
for f in dir bkt; do
  COP_BKT_XBITS=1 step 200 "$out/imix_${f}.log" python3 -u $R/bench.py --workload fw_lpm_imix --steps 1024 --warmup 256 --no-cpu --secondary none --route-form $f
  grep -h '^{"metric"' "$out/imix_${f}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], d["value"], "frac", r["frac"], "frac_timed", r.get("frac_timed"))' "imix_$f"
done
P="$R/bench.py --workload fw_lpm --steps 64 --warmup 16 --engine launch --no-cpu --secondary none"
for f in dir bkt; do
  step 200 "$out/pmc_${f}_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/${f}_fetch" -o bench --output-format csv -- python3 $P --route-form $f
  step 200 "$out/pmc_${f}_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/${f}_write" -o bench --output-format csv -- python3 $P --route-form $f
  step 200 "$out/pmc_${f}_hit.log" rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/${f}_hit" -o bench --output-format csv -- python3 $P --route-form $f
done
step 200 "$out/mb_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$out/mb_fetch" -o mb --output-format csv -- "$R/tools/membench"
step 200 "$out/mb_write.log" rocprofv3 --pmc WRITE_SIZE -d "$out/mb_write" -o mb --output-format csv -- "$R/tools/membench"
echo done
