#!/usr/bin/env bash
# Build librtg_hip.so from the csrc/ + include/ of a git revision into humanoid-real-time-retarget_amd/variants/<name>.so
# (the A/B base for tools/ab_headline.py: same box, same session, interleaved).  Build container only.
# usage: tools/build_rev.sh <rev> <name> [extra hipcc flags]
set -eu
rev=$1; name=$2; shift 2
repo="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$repo" archive "$rev" humanoid-real-time-retarget_amd/csrc include | tar -x -C "$tmp"
cd "$tmp/humanoid-real-time-retarget_amd/csrc"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -I../../include $*"
objs=""
# the revision's own TU list and per-TU flags (rtg_solve_fbp_small exists from round 5 on, with SMALL_FLAGS)
for f in rtg_*.hip; do
  t=${f%.hip}
  extra=""; { [ "$t" = rtg_solve_fbp_small ] || [ "$t" = rtg_fk ]; } && extra="-mllvm -amdgpu-sched-strategy=max-ilp"
  /opt/rocm/bin/hipcc $FLAGS $extra -c $t.hip -o $t.o &
  objs="$objs $t.o"
done
/opt/rocm/bin/hipcc $FLAGS -x hip -c rtg_api.cpp -o rtg_api.o &
wait
mkdir -p "$repo/humanoid-real-time-retarget_amd/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs rtg_api.o -o "$repo/humanoid-real-time-retarget_amd/variants/$name.so"
rm -rf "$tmp"
echo "built variants/$name.so from $rev"
