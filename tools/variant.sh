#!/bin/bash
# Builds an A/B variant of the library into bzip2_amd/var/<name>/ with extra compiler flags
# (development tool):  tools/variant.sh <name> "-DFOO=1 ..."
# then run with BZ2_AMD_LIB=bzip2_amd/var/<name>/libbz2_amd.so
set -e
cd "$(dirname "$0")/../bzip2_amd"
D=var/$1
mkdir -p $D
HIPCC=/opt/rocm/bin/hipcc
pids=()
for f in csrc/*.hip; do
  $HIPCC -O3 -std=c++17 -fPIC -Wno-unused-function --offload-arch=gfx950 $2 -c $f -o $D/$(basename $f .hip).o &
  pids+=($!)
done
for f in csrc/*.cpp; do
  $HIPCC -O2 -std=c++17 -fPIC -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $2 -c $f -o $D/$(basename $f .cpp).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -Wl,-soname,libbz2.so.1.0 -o $D/libbz2_amd.so $D/*.o
rm -f $D/*.o
