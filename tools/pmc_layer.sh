#!/bin/bash
# PMC anatomy of ONE conv layer under several forced engine configs (tools/one_layer.py --variant):
#   tools/pmc_layer.sh OUTDIR "COUNTERS" "ONE_LAYER_ARGS" v1 v2 ...
# one rocprofv3 --pmc pass per variant (each under its own time limit); parse with tools/pmc_layer.py.
set -e
out=$1; counters=$2; args=$3; shift 3
mkdir -p "$out"
export TMPDIR=/tmp
for v in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $counters -d "$out/v$v" -o p --output-format csv -- \
    python tools/one_layer.py $args --variant $v --reps 5 > "$out/v$v.log" 2>&1
  tail -n 1 "$out/v$v.log"
done
