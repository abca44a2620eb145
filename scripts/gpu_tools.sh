#!/bin/bash
# Development micro-benchmarks in build_tools/ (each under its own limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for f in build_tools/*; do
  [ -x "$f" ] || continue
  for a in ${TOOL_ARGS:-"1000000 0" "1000000 1"}; do
    echo "== $f $a"
    timeout -k 5 60 $f $a || { echo "FAIL $f"; exit 1; }
  done
done
