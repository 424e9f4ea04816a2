#!/bin/bash
# Builds an experimental variant of the library: tools_variant.sh NAME "-DFLAG=..." [sources to rebuild]
# -> variants/NAME.so (objects of unlisted sources are taken from bzip2_amd/build)
set -e
N=$1; F=$2; shift 2
cd /root/repo/bzip2_amd
mkdir -p ../variants build_var/$N
for o in scan rle1 sort sortdbl mtf code magic engine tieorder bzlib_api bzfile decode decomp; do cp -f build/$o.o build_var/$N/; done
for s in ${@:-sort}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 $F -c csrc/$s.hip -o build_var/$N/$s.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -Wl,-soname,libbz2.so.1.0 -o ../variants/$N.so build_var/$N/*.o
echo "variants/$N.so"
