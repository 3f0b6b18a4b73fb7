#!/bin/bash
# Builds libgtsfm_hip variants of ONE source file (extra -D flags) into build_var/ for A/B timing via GTSFM_HIP_LIB.
# Usage: build_variants_src.sh <file.hip> name1:"-DFOO=1" name2:"-DBAR" ...
set -e
cd "$(dirname "$0")/.."
SRC=$1; shift
B=$(basename $SRC .hip)
make -C gtsfm_amd/csrc -j8 >/dev/null
mkdir -p ${VARDIR:=build_var}
OBJS=$(ls gtsfm_amd/_lib/obj/*.o | grep -v "/$B.o")
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Igtsfm_amd/csrc $flags -c gtsfm_amd/csrc/$B.hip -o $VARDIR/${B}_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $VARDIR/libgtsfm_hip_$name.so $OBJS $VARDIR/${B}_$name.o
  echo "built $VARDIR/libgtsfm_hip_$name.so ($flags)"
done
