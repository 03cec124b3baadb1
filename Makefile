# MI355X k-mer engine.  `make` builds, as the reference's makefile does, a
# ./findKmer in this directory (findKmer/makefile:5-10), plus:
#   findkmer_amd/lib/libfindkmer_hip.so   C-ABI engine (include/findkmer.h)
#   Debug/findKmer                        same binary, for k6thru11fullANDupstream.sh
#   oracle/liboracle.so, oracle/_ref/     test checkers (never linked by the product)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXX      ?= g++
ROOT     := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
CSRC     := $(ROOT)findkmer_amd/csrc
LIBDIR   := $(ROOT)findkmer_amd/lib
BUILD    := $(ROOT)build
LIB      := $(LIBDIR)/libfindkmer_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -I$(ROOT)include -I$(CSRC) \
            -Wall -Wno-unused-function -Wno-unused-value -munsafe-fp-atomics
# the writer must evaluate long double / double exactly like the reference:
# plain g++, no fast-math, no FMA contraction
WFLAGS   := -O2 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -I$(ROOT)include -Wall

all: $(LIB) $(ROOT)findKmer $(ROOT)Debug/findKmer oracle

# the engine's translation units (one per path: state pass and k <= 7, the
# partition for 8 <= k <= 16, the sparse passes, the multi-GPU exchange, and
# the engine core / C-ABI) share fk_engine_internal.h
ENGINE_H := $(CSRC)/fk_engine_internal.h $(CSRC)/fk_part_kern.h $(CSRC)/fk_tiles.h $(CSRC)/fk_part.h $(CSRC)/fk_device.h \
            $(CSRC)/fk_sparse.h $(CSRC)/fk_comm.h $(ROOT)include/findkmer.h
ENGINE_TUS := fk_engine fk_scan fk_part fk_part_pipe fk_part_res fk_sparse_pass fk_exchange
ENGINE_OBJS := $(patsubst %,$(BUILD)/%.o,$(ENGINE_TUS))

$(ENGINE_OBJS): $(BUILD)/%.o: $(CSRC)/%.hip $(ENGINE_H)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -x hip $< -o $@

$(BUILD)/fk_writer.o: $(CSRC)/fk_writer.cpp $(ROOT)include/findkmer.h
	@mkdir -p $(BUILD)
	$(CXX) $(WFLAGS) -c $< -o $@

$(BUILD)/fk_sparse.o: $(CSRC)/fk_sparse.hip $(CSRC)/fk_sparse.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -x hip $< -o $@

$(BUILD)/fk_comm.o: $(CSRC)/fk_comm.hip $(CSRC)/fk_comm.h $(ROOT)include/findkmer.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -x hip $< -o $@

$(BUILD)/fk_ingest.o: $(CSRC)/fk_ingest.hip $(ROOT)include/findkmer.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -x hip $< -o $@

$(LIB): $(ENGINE_OBJS) $(BUILD)/fk_sparse.o $(BUILD)/fk_ingest.o $(BUILD)/fk_comm.o $(BUILD)/fk_writer.o
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread -ldl

$(BUILD)/fk_main.o: $(CSRC)/fk_main.cpp $(ROOT)include/findkmer.h
	@mkdir -p $(BUILD)
	$(CXX) $(WFLAGS) -c $< -o $@

$(ROOT)findKmer: $(BUILD)/fk_main.o $(LIB)
	$(CXX) -o $@ $(BUILD)/fk_main.o -L$(LIBDIR) -lfindkmer_hip -Wl,-rpath,'$$ORIGIN/findkmer_amd/lib' -lpthread

$(ROOT)Debug/findKmer: $(BUILD)/fk_main.o $(LIB)
	@mkdir -p $(ROOT)Debug
	$(CXX) -o $@ $(BUILD)/fk_main.o -L$(LIBDIR) -lfindkmer_hip -Wl,-rpath,'$$ORIGIN/../findkmer_amd/lib' -lpthread

oracle:
	$(MAKE) -C $(ROOT)oracle

clean:
	rm -rf $(BUILD) $(LIB) $(ROOT)findKmer $(ROOT)Debug

.PHONY: all oracle clean
