#!/bin/bash
# Same-box A/B of the MFMA Gram: tools/gram_probe.py in this tree and in abtest/<variant>, alternately.
# usage: tools/gram_ab.sh <variant> [rounds=2]
set -o pipefail
var="$1"; rounds="${2:-2}"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
for i in $(seq "$rounds"); do
  for T in "$R" "$R/abtest/$var"; do
    echo "== $(basename "$T")"
    timeout -k 10 200 python3 "$T/tools/gram_probe.py" 3 || exit $?
  done
done
