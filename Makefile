# Build libminehip.so (gfx950 HIP kernels + C-ABI) and the CPU oracle.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := bitcoin-miner_amd
CSRC    := $(PKG)/csrc
LIB     := $(PKG)/minehip/libminehip.so
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRCS    := $(CSRC)/search_kernels.hip $(CSRC)/minehip.cpp $(CSRC)/plan.cpp $(CSRC)/message.cpp
HDRS    := $(CSRC)/layout.hpp $(CSRC)/plan.hpp $(CSRC)/sha256_gfx950.hpp include/minehip.h

all: $(LIB) oracle

$(LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

oracle:
	$(MAKE) -s -C oracle

# disassembly + register report of the kernels (for DESIGN.md / profiling)
asm: $(SRCS) $(HDRS)
	mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/search_kernels.s $(CSRC)/search_kernels.hip

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle asm clean
