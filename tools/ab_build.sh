#!/bin/bash
# Build librf_amd from a git revision into tools/ab/librf_amd_<tag>.so (A/B experiments).
# usage: [AB_PATCH=f] tools/ab_build.sh <rev> <tag> ["-DMACRO=V ..."]   (rev WT = the working tree)
set -e
REV=$1; TAG=$2; DEFS=$3; D=$(mktemp -d)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $D/splinterdb_amd/csrc $D/include
for f in splinterdb_amd/csrc/rf_kernels.hip splinterdb_amd/csrc/rf_engine.cpp splinterdb_amd/csrc/rf_device.h splinterdb_amd/csrc/rf_plan.h include/rf_amd.h include/rf_amd_diag.h; do
  if [ "$REV" = WT ]; then cp $ROOT/$f $D/$f; else git -C $ROOT show $REV:$f > $D/$f; fi
done
# AB_PATCH=<file>: a patch (git diff from the repo root) applied to the copied sources
if [ -n "$AB_PATCH" ]; then patch -s -d $D -p1 < $AB_PATCH; fi
H=/opt/rocm/bin/hipcc
# the working tree's build id (a variant of the tree's sources loads through engine.py's check;
# AB_TREE_ID=1 gives a revision's build the same id)
if [ "$REV" = WT ] || [ -n "$AB_TREE_ID" ]; then DEFS="$DEFS -DRF_AMD_SRC_ID=\"$(cd $ROOT && python3 -c 'from splinterdb_amd import build; print(build.source_id())')\""; fi
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC $DEFS -c $D/splinterdb_amd/csrc/rf_kernels.hip -o $D/k.o
$H -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC $DEFS -c $D/splinterdb_amd/csrc/rf_engine.cpp -o $D/e.o
$H --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/ab/librf_amd_$TAG.so $D/k.o $D/e.o
rm -rf $D
echo built tools/ab/librf_amd_$TAG.so
