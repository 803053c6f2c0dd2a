# Build everything the hot path needs (gfx950 only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall
CSRC := p1_amd/csrc
HDRS := $(CSRC)/sha256_dev.hpp $(CSRC)/scan_core.hpp $(CSRC)/planner.hpp $(CSRC)/fast_variants.inc include/p1hip.h

all: p1_amd/libp1hip.so oracle tools/p1emu p1_amd/p1miner p1_amd/p1server

p1_amd/libp1hip.so: $(CSRC)/p1hip.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/p1hip.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# C++ host mirror of the reference's bitcoin package + miner loop (stdio)
p1_amd/p1miner: p1_amd/host/p1miner.cpp p1_amd/host/bitcoin.cpp p1_amd/host/bitcoin.hpp include/p1hip.h p1_amd/libp1hip.so
	g++ -O2 -std=c++17 -Wall -Wextra -o $@ p1_amd/host/p1miner.cpp p1_amd/host/bitcoin.cpp -Lp1_amd -lp1hip -Wl,-rpath,'$$ORIGIN'

p1_amd/p1server: p1_amd/host/p1server.cpp p1_amd/host/bitcoin.cpp p1_amd/host/bitcoin.hpp include/p1hip.h p1_amd/libp1hip.so
	g++ -O2 -std=c++17 -Wall -Wextra -o $@ p1_amd/host/p1server.cpp p1_amd/host/bitcoin.cpp -Lp1_amd -lp1hip -Wl,-rpath,'$$ORIGIN'

# host-only replay of the kernels' per-thread code (layout tests; not product)
tools/p1emu: tools/p1emu.cpp $(HDRS)
	$(HIPCC) -O2 -std=c++17 -o $@ tools/p1emu.cpp

oracle:
	$(MAKE) -C oracle

# A/B tuning builds (not used unless P1HIP_LIB points at one)
variants: p1_amd/variants/libp1hip_w4.so p1_amd/variants/libp1hip_w6.so p1_amd/variants/libp1hip_w8.so
p1_amd/variants/libp1hip_w%.so: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p p1_amd/variants
	$(HIPCC) $(HIPFLAGS) -DP1_FAST_WAVES=$* -shared -o $@ $(CSRC)/p1hip.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# ISA + resource report of the scan kernels (for DESIGN.md / profiling)
isa: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p build/isa && cd build/isa && $(HIPCC) $(HIPFLAGS) -c ../../$(CSRC)/p1hip.hip -o p1hip.o -save-temps -Rpass-analysis=kernel-resource-usage 2> resource.txt

clean:
	rm -f p1_amd/libp1hip.so tools/p1emu p1_amd/p1miner p1_amd/p1server
	$(MAKE) -C oracle clean
.PHONY: all oracle clean isa variants
