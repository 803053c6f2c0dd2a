# Build everything the hot path needs (gfx950 only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall
CSRC := p1_amd/csrc
HDRS := $(CSRC)/sha256_dev.hpp $(CSRC)/scan_core.hpp $(CSRC)/planner.hpp $(CSRC)/fast_variants.inc include/p1hip.h

all: p1_amd/libp1hip.so oracle tools/p1emu

p1_amd/libp1hip.so: $(CSRC)/p1hip.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/p1hip.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# host-only replay of the kernels' per-thread code (layout tests; not product)
tools/p1emu: tools/p1emu.cpp $(HDRS)
	$(HIPCC) -O2 -std=c++17 -o $@ tools/p1emu.cpp

oracle:
	$(MAKE) -C oracle

# ISA + resource report of the scan kernels (for DESIGN.md / profiling)
isa: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p build/isa && cd build/isa && $(HIPCC) $(HIPFLAGS) -c ../../$(CSRC)/p1hip.hip -o p1hip.o -save-temps -Rpass-analysis=kernel-resource-usage 2> resource.txt

clean:
	rm -f p1_amd/libp1hip.so tools/p1emu
	$(MAKE) -C oracle clean
.PHONY: all oracle clean isa
