#!/bin/bash
# Interleaved A/B of environment settings over one command (separate processes, so settings read
# once per process -- HH_FUSED_ROWS, HH_BASIS_PAD, HH_LIB_PATH -- can be compared):
#   tools/ab_env.sh REPS "ENV_A" "ENV_B" ... -- CMD ARGS
# prints each run's "it/s" lines, or for a bench.py JSON line its SpMV value and GMRES rates,
# prefixed by the setting.
set -u
REPS=$1; shift
SETS=()
while [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
summ() { python3 "$(dirname "$0")/ab_summ.py" "$1"; }
for r in $(seq 1 "$REPS"); do
  for s in "${SETS[@]}"; do
    out=$(env $s timeout -k 10 300 "$@" 2>&1) || { echo "[$s] FAILED rc=$?"; echo "$out" | tail -5; exit 1; }
    echo "$out" | summ "$s"
  done
done
