#!/bin/bash
# Build an alternative libemurx.so with extra compiler flags, for A/B runs (EMURX_LIB=...):
#   tools/build_variant.sh <name> "<-DFLAG=..>"   -> trex-emu_amd/lib/libemurx_<name>.so
set -eu
cd "$(dirname "$0")/../trex-emu_amd"
name=$1; flags=$2
out=build/var_$name
mkdir -p $out lib
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags"
objs=""
for f in emurx_kernels emurx_route emurx_ingest emurx_tx emurx_txzmq; do
  /opt/rocm/bin/hipcc $F -c csrc/$f.hip -o $out/$f.o &
  objs="$objs $out/$f.o"
done
/opt/rocm/bin/hipcc $F -x hip -c csrc/emurx_api.cpp -o $out/emurx_api.o &
/opt/rocm/bin/hipcc $F -c csrc/emurx_comm.cpp -o $out/emurx_comm.o &
${CXX:-g++} -O2 -std=c++17 -fPIC -Wall $flags -c csrc/emurx_mirror.cpp -o $out/emurx_mirror.o &
wait
make -s build/build_id.o
/opt/rocm/bin/hipcc $F -shared -o lib/libemurx_$name.so $objs $out/emurx_api.o $out/emurx_mirror.o $out/emurx_comm.o \
  build/build_id.o -ldl
echo lib/libemurx_$name.so
