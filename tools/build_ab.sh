#!/bin/bash
# A/B library builds (tooling): lib/libslatecodec_<tag>.so = the current objects with the
# decode kernel compiled from SRC (e.g. a git revision's decode_lpb2.hip) and extra FLAGS, built
# exactly as the Makefile builds the shipped library (no profiling switches).
# usage: tools/build_ab.sh TAG SRC.hip ["FLAGS"]   env: OBJ (the object SRC replaces, default
# decode_lpb2; its scheduler flag SCHED applies to decode_lpb2 only)
set -e
TAG=$1; SRC=$(realpath "$2"); FLAGS=$3; OBJ=${OBJ:-decode_lpb2}
if [ "$OBJ" != decode_lpb2 ]; then SCHED=${SCHED-}; fi
cd "$(dirname "$0")/../slatedb-go_amd"
make -s
mkdir -p build/ab_$TAG
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-parameter"
/opt/rocm/bin/hipcc $HIPFLAGS ${SCHED--mllvm -amdgpu-sched-strategy=max-ilp} -Icsrc $FLAGS -c "$SRC" -o build/ab_$TAG/$OBJ.hip.o
objs=$(ls build/*.o | grep -v "/$OBJ.hip.o")
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o lib/libslatecodec_$TAG.so $objs build/ab_$TAG/$OBJ.hip.o
echo lib/libslatecodec_$TAG.so
