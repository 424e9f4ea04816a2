#!/bin/bash
# Builds the library of git revision REV (sources only, this tree's build flags) as
# variants/NAME.so, for same-box A/B runs against the working tree (development tool):
#   tools_ab_rev.sh REV NAME
set -e
REV=$1; N=$2
T=/tmp/abrev_$N; rm -rf $T; mkdir -p $T/bzip2_amd/csrc $T/include $T/obj
cd /root/repo
for f in $(git ls-tree --name-only -r $REV bzip2_amd/csrc); do git show $REV:$f > $T/bzip2_amd/csrc/$(basename $f); done
for f in include/bzg.h include/bzlib.h; do git show $REV:$f > $T/include/$(basename $f); done
pids=()
for f in $T/bzip2_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -I$T/include -c $f -o $T/obj/$(basename $f .hip).o & pids+=($!)
done
for f in $T/bzip2_amd/csrc/*.cpp; do
  /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Wall -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$T/include -c $f -o $T/obj/$(basename $f .cpp).o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -Wl,-soname,libbz2.so.1.0 -o variants/$N.so $T/obj/*.o
echo variants/$N.so
