#!/bin/bash
# k_part variants: build/exp/libfk_pw<W>.so with PART_WAVES=W (the product
# build uses the default in fk_engine.hip); load one with FINDKMER_LIB=...
set -e
cd "$(dirname "$0")/.."
mkdir -p build/exp
for w in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-unused-value \
    -Iinclude -Ifindkmer_amd/csrc -DPART_WAVES=${w}u -c -o build/exp/pw$w.o findkmer_amd/csrc/fk_engine.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/exp/libfk_pw$w.so build/exp/pw$w.o build/fk_sparse.o \
    build/fk_ingest.o build/fk_writer.o -lpthread
done
