#!/bin/bash
# A/B of the driver's 20-step command under environment variants (poll-mode
# knobs): each variant runs bench.py --quick with 21 timed runs; prints the
# median line. usage: tools/ab20.sh <outdir> "NAME:ENV=V ENV2=V" ...
set -o pipefail
out=$1; shift
mkdir -p "$out"
for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    [ "$envs" = "$name" ] && envs=""
    env $envs timeout -k 10 200 python3 bench.py --quick --steps 20 --warmup 5 --repeats 21 > "$out/$name.log" 2>&1 || exit 1
    python3 tools/summ.py "$out/$name.log" | head -1
done
