#!/bin/bash
# Build the library of git revision $1 into build_abl/lib_$2.so (A/B baseline
# for scripts/gpu.sh ab). Uses a temporary worktree; the tree here is untouched.
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
wt=$(mktemp -d /tmp/rlref.XXXXXX)
git -C "$root" worktree add -q --detach "$wt" "$rev"
(cd "$wt" && python -m ratelimit_amd.build --force > /dev/null)
mkdir -p "$root/build_abl"
cp "$wt/ratelimit_amd/libratelimit_hip.so" "$root/build_abl/lib_$name.so"
git -C "$root" worktree remove --force "$wt"
echo "$root/build_abl/lib_$name.so"
