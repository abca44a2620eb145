#!/bin/bash
# Development micro-benchmarks in build_tools/ (each under its own limit).
# TOOL_ARGS: ';'-separated argument lists.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
IFS=';' read -ra SETS <<< "${TOOL_ARGS:-1000000 0;1000000 1}"
for f in build_tools/*; do
  [ -x "$f" ] || continue
  for a in "${SETS[@]}"; do
    echo "== $f $a"
    timeout -k 5 60 $f $a || { echo "FAIL $f"; exit 1; }
  done
done
