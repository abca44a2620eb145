#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for f in build_tools/sortbench_*; do timeout -k 5 60 $f 1000000 || { echo "FAIL $f"; exit 1; }; done
