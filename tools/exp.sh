#!/bin/bash
# Ablation variants of the engine library (k_count experiments only; the
# product build is FK_EXP=0).  Output: build/exp/libfk_e<N>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/exp
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-unused-value \
    -Iinclude -Ifindkmer_amd/csrc -DFK_EXP=$n -c -o build/exp/e$n.o findkmer_amd/csrc/fk_engine.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/exp/libfk_e$n.so build/exp/e$n.o build/fk_sparse.o build/fk_ingest.o build/fk_comm.o build/fk_writer.o -lpthread -ldl
done
