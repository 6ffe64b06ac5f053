# Build everything in-tree (the .so / binaries travel to the GPU box with the
# gpurun snapshot; they are git-ignored).
#   libphj_hip.so : HIP kernels + C ABI (include/phj.h), gfx950 only
#   phjoin        : the reference-compatible CLI (C++ host driver over the C ABI)
#   oracle        : CPU restatement (test infrastructure) + oracle/_ref when the
#                   reference sources are mounted
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
PKG := partitionedhashjoin_amd
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
CXXFLAGS := -std=c++17 -O2 -Wall -Wextra -pthread -ffp-contract=off

LIB := $(PKG)/libphj_hip.so
CLI := $(PKG)/phjoin
HIP_SRC := $(PKG)/csrc/phj_capi.hip
HIP_HDR := $(PKG)/csrc/phj_table.h $(PKG)/csrc/phj_pow.h $(PKG)/csrc/phj_pow_tables.h $(PKG)/csrc/phj_group.h $(PKG)/csrc/phj_partition.h $(PKG)/csrc/phj_join.h $(PKG)/csrc/phj_mat.h $(PKG)/csrc/phj_hash.h include/phj.h
HOST_SRC := $(wildcard $(PKG)/host/*.cpp $(PKG)/host/*/*.cpp)
HOST_HDR := $(wildcard $(PKG)/host/*.hpp $(PKG)/host/*/*.hpp) $(PKG)/csrc/phj_hash.h

ifneq ($(HOST_SRC),)
all: $(LIB) $(CLI) oracle

lib: $(LIB)
else
all: $(LIB) oracle
endif

$(LIB): $(HIP_SRC) $(HIP_HDR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRC)

$(CLI): $(HOST_SRC) $(HOST_HDR) include/phj.h $(LIB)
	$(CXX) $(CXXFLAGS) -Iinclude -I$(PKG)/host -I$(PKG)/csrc -o $@ $(HOST_SRC) -L$(PKG) -lphj_hip -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -s -C oracle liboracle.so
	@if [ -d /root/reference/src ]; then $(MAKE) -s -C oracle/ref; fi

clean:
	rm -f $(LIB) $(CLI)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean lib
