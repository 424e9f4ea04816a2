#!/bin/bash
# Builds the library of a git revision into bzip2_amd/var/<name>/ (development A/B tool):
#   tools/var_ref.sh <name> <rev> ["-DFOO=1 ..."]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$2" bzip2_amd/csrc bzip2_amd/Makefile include | tar -x -C "$T"
D=$ROOT/bzip2_amd/var/$1
mkdir -p "$D"
make -s -j8 -C "$T/bzip2_amd" CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 $3" libbz2_amd.so
cp "$T/bzip2_amd/libbz2_amd.so" "$D/libbz2_amd.so"
rm -rf "$T"
