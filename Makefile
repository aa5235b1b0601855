# Build libminehip.so (gfx950 HIP kernels + C-ABI) and the CPU oracle.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := bitcoin-miner_amd
CSRC    := $(PKG)/csrc
LIB     := $(PKG)/minehip/libminehip.so
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRCS    := $(CSRC)/search_kernels.hip $(CSRC)/minehip.cpp $(CSRC)/plan.cpp $(CSRC)/multi.cpp $(CSRC)/message.cpp \
           $(CSRC)/sched.cpp $(CSRC)/server.cpp
HDRS    := $(CSRC)/layout.hpp $(CSRC)/plan.hpp $(CSRC)/sha256_gfx950.hpp $(CSRC)/msgcodec.hpp \
           $(CSRC)/sched.hpp $(CSRC)/multi.hpp $(CSRC)/kernel_common.hpp include/minehip.h include/minehip_server.h
LLVM    ?= /opt/rocm/lib/llvm/bin
BUILD   := build
FAST_HDRS := $(CSRC)/kernel_common.hpp $(CSRC)/layout.hpp $(CSRC)/sha256_gfx950.hpp
FAST_S  := $(BUILD)/fast_search.s
FAST_SP := $(BUILD)/fast_search_split.s
FAST_PS := $(BUILD)/fast_search_prio.s
FAST_MIX := $(BUILD)/fast_loop_mix.json
# every ADD3_SPLIT-th v_add3 of each fast kernel as two full-rate adds (csrc/add3_split.py; 0: none)
ADD3_SPLIT ?= 3
FAST_CO := $(BUILD)/fast_search.hsaco
FAST_O  := $(BUILD)/fast_co.o
FASTFLAGS ?=

LSPLIB  := $(PKG)/minehip/liblsp440.so
APPS    := $(CSRC)/apps
BIN     := $(PKG)/bin
CLIS    := $(BIN)/minehip-search $(BIN)/minehip-miner $(BIN)/minehip-server $(BIN)/minehip-client
RPATH   := -Wl,-rpath,'$$ORIGIN/../minehip'

DEVLIB  := $(BUILD)/dev/libminehip.so

all: $(LIB) $(LSPLIB) $(CLIS) oracle dev $(BUILD)/libclockprobe.so $(BUILD)/libvaluenergy.so $(FAST_MIX) $(BUILD)/fast_search_nomarker.hsaco

# LSP endpoint (host only, wire compatible with the reference's Go lsp package)
$(LSPLIB): $(CSRC)/lsp/lsp.cpp include/lsp440.h
	g++ -O2 -std=c++17 -Wall -Wextra -fPIC -shared -o $@ $(CSRC)/lsp/lsp.cpp -lpthread

$(LIB): $(SRCS) $(HDRS) $(FAST_O)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS) -x none $(FAST_O)

# dev build: the same library plus the experiment / test hooks (MINEHIP_DEV_CODE_OBJECT,
# MINEHIP_DEV_LDS, MINEHIP_TEST_FAIL_WORKER, MINEHIP_TEST_SPAWN_LIMIT).  Never the package's library: tools and the
# tests that need a hook load it explicitly (MINEHIP_LIB=build/dev/libminehip.so).
dev: $(DEVLIB)
$(DEVLIB): $(SRCS) $(HDRS) $(FAST_O)
	mkdir -p $(BUILD)/dev
	$(HIPCC) $(HIPFLAGS) -DMH_DEV_HOOKS -shared -o $@ $(SRCS) -x none $(FAST_O)

# fast_search<J, MODE>: gfx950 assembly -> add3 split (every third v_add3 as two full-rate adds)
# -> issue-priority pass (s_setprio around half-/full-rate runs) -> code object ->
# embedded in the library (fast_co.S); the per-nonce loops' issued mix -> fast_loop_mix.json (bench)
$(FAST_S): $(CSRC)/fast_search.hip $(FAST_HDRS)
	mkdir -p $(BUILD)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) $(FASTFLAGS) --cuda-device-only -S -o $@ $<
# the split factor is a prerequisite: `make ADD3_SPLIT=k` after a build redoes the split (and the
# loop mix bench.py reads) instead of reusing the old assembly
ADD3_STAMP := $(BUILD)/add3_split.$(ADD3_SPLIT).stamp
$(ADD3_STAMP):
	mkdir -p $(BUILD)
	rm -f $(BUILD)/add3_split.*.stamp
	touch $@
$(FAST_SP): $(FAST_S) $(CSRC)/add3_split.py $(ADD3_STAMP)
	python3 $(CSRC)/add3_split.py $(ADD3_SPLIT) $< $@
$(FAST_PS): $(FAST_SP) $(CSRC)/issue_prio.py $(CSRC)/valu_rates.py
	python3 $(CSRC)/issue_prio.py $< $@
$(FAST_MIX): $(FAST_PS) $(CSRC)/loop_mix.py $(CSRC)/valu_rates.py
	python3 $(CSRC)/loop_mix.py $< $@
$(FAST_CO): $(FAST_PS)
	$(LLVM)/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=$(ARCH) -c -o $(BUILD)/fast_search_prio.o $<
	$(LLVM)/ld.lld -shared -o $@ $(BUILD)/fast_search_prio.o
# test artefact: the same kernels without the work-queue marker (mh_fast_queue_args), as a code
# object built from older sources would be; the dev build must run it one workgroup per chunk
# (tests/test_gpu_parity.py::test_code_object_without_queue_marker_runs_static)
$(BUILD)/fast_search_nomarker.hsaco: $(FAST_PS)
	grep -v mh_fast_queue_args $< > $(BUILD)/fast_search_nomarker.s
	$(LLVM)/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=$(ARCH) -c -o $(BUILD)/fast_search_nomarker.o $(BUILD)/fast_search_nomarker.s
	$(LLVM)/ld.lld -shared -o $@ $(BUILD)/fast_search_nomarker.o
$(FAST_O): $(CSRC)/fast_co.S $(FAST_CO)
	gcc -c -fPIC -Wa,-I,$(BUILD) -o $@ $<

# native C++ callers of the C-ABI (rpath: the library next to the package)
$(BIN)/minehip-search: $(CSRC)/cli.cpp include/minehip.h $(LIB)
	mkdir -p $(BIN)
	g++ -O2 -std=c++17 -Wall -o $@ $(CSRC)/cli.cpp -L$(PKG)/minehip -lminehip $(RPATH)

# miner / server / client processes over LSP (bitcoin/{miner,server,client})
$(BIN)/minehip-%: $(APPS)/%_main.cpp $(APPS)/common.hpp include/minehip.h include/minehip_server.h include/lsp440.h $(LIB) $(LSPLIB)
	mkdir -p $(BIN)
	g++ -O2 -std=c++17 -Wall -Wextra -o $@ $< -L$(PKG)/minehip -lminehip -llsp440 $(RPATH) -lpthread

oracle:
	$(MAKE) -s -C oracle

# in-kernel clock probe (measurement only: bench.py's roofline.kernel_clock)
$(BUILD)/libclockprobe.so: tools/clock_probe.hip
	mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# energy per VALU instruction class at the power limit (measurement only: tools/energy_probe.py)
$(BUILD)/libvaluenergy.so: tools/valu_energy.hip
	mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# disassembly + register report of the kernels (for DESIGN.md / profiling)
asm: $(FAST_PS)
	mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/search_kernels.s $(CSRC)/search_kernels.hip

# VALU issue-rate microbenchmarks, run by tools/gpu_session.sh
probes: build/valu_peak build/valu_ops build/valu_mix build/valu_pair build/valu_bank
build/valu_bank: tools/gen_valu_bank.py
	mkdir -p build
	python3 tools/gen_valu_bank.py
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ tools/valu_bank.hip
build/valu_pair: tools/gen_valu_pair.py
	mkdir -p build
	python3 tools/gen_valu_pair.py
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ tools/valu_pair.hip
build/valu_mix: tools/gen_valu_mix.py
	mkdir -p build
	python3 tools/gen_valu_mix.py
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ tools/valu_mix.hip
build/valu_%: tools/valu_%.hip
	mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

clean:
	rm -f $(LIB) $(DEVLIB) $(LSPLIB) $(CLIS) $(FAST_S) $(FAST_SP) $(FAST_PS) $(FAST_MIX) $(FAST_CO) $(FAST_O) \
	      $(BUILD)/fast_search_prio.o $(BUILD)/libclockprobe.so $(BUILD)/libvaluenergy.so $(BUILD)/add3_split.*.stamp \
	      $(BUILD)/fast_search_nomarker.*
	$(MAKE) -s -C oracle clean

.PHONY: all oracle asm clean probes dev
