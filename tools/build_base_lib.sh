#!/bin/bash
# Build libhmcx.so of another commit (default: the round-2 closing commit) into
# dropout_hamiltonian_montecarlo_amd/lib/libhmcx_<tag>.so for same-box A/B runs (HMCX_LIB=...).
# Usage: bash tools/build_base_lib.sh [commit] [tag]
set -e
C=${1:-3a776b3}; TAG=${2:-r02}
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/hmcx_wt_$TAG
rm -rf $W; git -C $R worktree prune; git -C $R worktree add -f --detach $W $C >/dev/null
S=$W/dropout_hamiltonian_montecarlo_amd/csrc
mkdir -p $W/obj
for f in $S/*.hip; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -I$W/include -I$S -c $f -o $W/obj/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/dropout_hamiltonian_montecarlo_amd/lib/libhmcx_$TAG.so $W/obj/*.o
git -C $R worktree remove --force $W
echo built libhmcx_$TAG.so from $C
