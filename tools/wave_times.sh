#!/bin/bash
# experiment build with per-wave timestamps in k_count: build/exp/libfk_wt.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-unused-value \
  -Iinclude -Ifindkmer_amd/csrc -DFK_WAVE_TIMES -c -o build/exp/wt.o findkmer_amd/csrc/fk_engine.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/exp/libfk_wt.so build/exp/wt.o build/fk_sparse.o \
  build/fk_ingest.o build/fk_writer.o -lpthread
