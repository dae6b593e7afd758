#!/bin/bash
# A/B of the one-launch reduction (default) against the two-stage one (PPLS_REDUCE_FUSED=0): C4 share
# and C5 share benches, interleaved.  Timing only.
set -o pipefail
for v in 1 0 1 0; do
  for cfg in c4s c5s; do
    echo "== fused=$v $cfg"
    PPLS_REDUCE_FUSED=$v timeout -k 10 120 python bench.py --config $cfg --no-cpu --steps 60 | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
