#!/bin/bash
# A/B of poll-mode variants on the driver's command plus the poll-mode
# steady state (bench.py without --quick, no CPU baseline, no secondary):
# usage: tools/ab_pmd.sh <outdir> "NAME:ENV=V ENV2=V" ...
set -o pipefail
out=$1; shift
mkdir -p "$out"
for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    [ "$envs" = "$name" ] && envs=""
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --repeats 11 --no-cpu --secondary none \
        > "$out/$name.log" 2>&1 || exit 1
    python3 - "$out/$name.log" "$name" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
r, p = d["roofline"], d.get("pmd", {})
print(f'{sys.argv[2]:10s} value {d["value"]:9.1f} frac_timed {r["frac_timed"]:.4f} frac {r["frac"]:.4f} '
      f'steady {p.get("steady_mpkt_s")} ({p.get("steady_frac")}) one-batch {p.get("single_batch_post_to_done_us_median")} us '
      f'16-in-flight {p.get("one_batch_posts", {}).get("mpkt_s")}')
PY
done
