#!/bin/bash
# Build tools/sortbench for several onesweep tile shapes (items x waves).
set -e
cd "$(dirname "$0")/.."
mkdir -p build_tools
for cfg in "16 4" "8 4" "8 8" "4 8" "16 8" "4 16"; do
  set -- $cfg
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iratelimit_amd/csrc \
    -DRL_OS_ITEMS=$1 -DRL_OS_WAVES=$2 tools/sortbench.hip -o build_tools/sortbench_$1_$2 &
done
wait
ls build_tools
