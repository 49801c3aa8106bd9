#!/bin/bash
# Experiment builds (tooling): libslatecodec_<tag>.so with extra compile flags on the
# decode kernel, selected at run time by SLATE_LIB_VARIANT=libslatecodec_<tag>.so.
# usage: tools/variant.sh TAG "-DSLATE_LPB_THREADS=512 -DSLATE_LPB_NS=8"
set -e
TAG=$1; FLAGS=$2
cd "$(dirname "$0")/../slatedb-go_amd"
make -s
mkdir -p build/var_$TAG
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-parameter -DSLATE_PROFILING_BUILD"
objs=""
for f in build/*.o; do
  b=$(basename $f)
  case $b in
    decode_lpb2.hip.o|decode.hip.o|decode_none.hip.o|zstd_fast.hip.o|api_sst.cpp.o|encode.hip.o|encode_codecs.hip.o)
      extra=""; [ $b = decode_lpb2.hip.o ] && extra="${LPB_SCHED--mllvm -amdgpu-sched-strategy=max-ilp}"  # as the Makefile (LPB_SCHED overrides)
      /opt/rocm/bin/hipcc $HIPFLAGS $extra $FLAGS -c csrc/${b%.o} -o build/var_$TAG/$b; objs="$objs build/var_$TAG/$b";;
    *) objs="$objs $f";;
  esac
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o lib/libslatecodec_$TAG.so $objs
echo lib/libslatecodec_$TAG.so
