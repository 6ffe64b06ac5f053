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
HIP_HDR := $(wildcard $(PKG)/csrc/*.h) include/phj.h
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

# measurement build (not shipped): the phase-clock forms of S's pass 1 and of
# the LDS join's builds (stderr per join); select it with PHJ_LIB=build/libphj_prof.so
prof-lib: build/libphj_prof.so
build/libphj_prof.so: $(HIP_SRC) $(HIP_HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DPHJ_P1_PROF=1 -DPHJ_CL_PROF=1 -shared -o $@ $(HIP_SRC)

# A/B variants of the same sources: make build/libphj_NAME.so HIPDEFS="-DPHJ_PIPE_RES=1"
build/libphj_%.so: $(HIP_SRC) $(HIP_HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(HIPDEFS) -shared -o $@ $(HIP_SRC)

oracle:
	$(MAKE) -s -C oracle liboracle.so
	@if [ -d /root/reference/src ]; then $(MAKE) -s -C oracle/ref; fi

clean:
	rm -f $(LIB) $(CLI)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean lib prof-lib
