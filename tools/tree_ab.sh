#!/bin/bash
# Steady-state A/B of experiment builds (abtest/<variant>, each a copy of the tree with its own
# libppls_amd.so) against the product: ms per EM iteration from tools/option_ab.py (back-to-back
# iterations, defaults), arms interleaved in separate processes on the same box.
# usage: tools/tree_ab.sh <config> <variant> [<variant> ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cfg="$1"; shift
for arm in base "$@" base "$@"; do
  if [ "$arm" = base ]; then T="$R"; else T="$R/abtest/$arm"; fi
  line=$(timeout -k 10 120 python3 "$T/tools/option_ab.py" "$cfg" "" --reps 2 --iters 40 | tail -1) || exit $?
  echo "$cfg $arm: $line"
done
