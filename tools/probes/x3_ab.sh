#!/bin/bash
# A/B of x3 probe builds (interleaved rounds in separate processes on one box):
#   tools/probes/x3_ab.sh <rounds> <so1> <so2> ... -- <x3_micro args>
set -e
rounds=$1; shift
sos=()
while [ "$1" != "--" ]; do sos+=("$1"); shift; done
shift
for r in $(seq 1 $rounds); do
  for so in "${sos[@]}"; do
    echo "== $so round $r"
    if [ "$so" = "default" ]; then
      timeout -k 10 200 python3 bench/x3_micro.py "$@"
    elif [ "${so#env:}" != "$so" ]; then
      env "${so#env:}" timeout -k 10 200 python3 bench/x3_micro.py "$@"
    elif [ "${so#tree:}" != "$so" ]; then
      (cd ${so#tree:} && PYTHONPATH=. timeout -k 10 200 python3 bench/x3_micro.py "$@")
    else
      APNEAUQ_SO_PATH=$so timeout -k 10 200 python3 bench/x3_micro.py "$@"
    fi
  done
done
