# Build everything the hot path needs (gfx950 only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall
LLVM ?= /opt/rocm/lib/llvm/bin
CSRC := p1_amd/csrc
HDRS := $(CSRC)/sha256_dev.hpp $(CSRC)/scan_core.hpp $(CSRC)/planner.hpp $(CSRC)/fast_variants.inc $(CSRC)/variant_cost.inc \
        $(CSRC)/scan_abi.hpp include/p1hip.h
# what the device code includes (the host-side planner does not rebuild it)
DEVHDRS := $(CSRC)/sha256_dev.hpp $(CSRC)/scan_core.hpp $(CSRC)/fast_variants.inc $(CSRC)/scan_abi.hpp
# device code: HIP C++ -> gfx950 assembly -> tools/isa_post.py post-pass
# (ISAPOST: LLVM's own encodings kept (--no-e64); loop labels aligned; every
# loop body's straight-line segments reordered into runs of one issue class
# (tools/pair_sched.py) with `s_setprio 1` / `s_setprio 0` before each
# half-rate / full-rate run; DESIGN.md 4 "Dual issue"; --strict-hazards: the
# build fails if a reorder would shorten a wait-state distance LLVM relied
# on, tools/pair_sched.py check_hazards) -> assembled + linked code object,
# embedded in libp1hip.so.
# -amdgpu-s-branch-bits=15: the post-pass inserts ~21.7k 4-byte s_setprio and
# the loop-alignment padding AFTER the compiler has relaxed its branches, so
# the compiler is told branches reach half their real range (+-2^14 of
# +-2^15 dwords) and a branch it leaves short still fits after the growth
# (shipped object: largest displacement 15,551 dwords; the long branches it
# expands are the variant dispatch's, outside every per-nonce loop).  A
# branch that did not fit would fail the assembly ("branch size exceeds
# simm16"), never build wrong code (tests/test_codeobj.py).
DEVFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) --cuda-device-only -Wall -mllvm -amdgpu-s-branch-bits=15 $(DEVEXTRA)
ISAPOST ?= --no-e64 --align-loops=3 --loop-offset=4 --pair-sched=0 --sched-amax=5 --sched-bmax=4 --strict-hazards --prio=0,1
BUILD := build

all: p1_amd/libp1hip.so oracle tools/p1emu p1_amd/p1miner p1_amd/p1server p1_amd/p1client tools/lsp_scenarios \
     tools/lsp_fake_miner tools/queue_ctl tools/wcal tools/vbank tools/libp1clock.so

# The assembly and object stages are intermediates: once the code object
# exists, a tree without them (the GPU box's copy leaves the 16 MB of .s out,
# .gpurunignore) does not recompile the kernels unless a source is newer.
.SECONDARY: $(BUILD)/p1hip_kernels.s $(BUILD)/p1hip_kernels.post.s $(BUILD)/p1hip_kernels.o
$(BUILD)/p1hip_kernels.s: $(CSRC)/p1hip_kernels.hip $(DEVHDRS) Makefile
	mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -S -o $@ $(CSRC)/p1hip_kernels.hip

$(BUILD)/p1hip_kernels.post.s: $(BUILD)/p1hip_kernels.s tools/isa_post.py tools/pair_sched.py
	python3 tools/isa_post.py $< $@ $(ISAPOST)

$(BUILD)/p1hip_kernels.o: $(BUILD)/p1hip_kernels.post.s
	$(LLVM)/clang -cc1as -triple amdgcn-amd-amdhsa -filetype obj -target-cpu $(ARCH) -mrelocation-model pic -o $@ $<

$(BUILD)/p1hip_kernels.hsaco: $(BUILD)/p1hip_kernels.o
	$(LLVM)/ld.lld -m elf64_amdgpu --no-undefined -shared -o $@ $<

$(BUILD)/p1hip_kernels_blob.o: $(CSRC)/p1hip_kernels_blob.S $(BUILD)/p1hip_kernels.hsaco
	gcc -c -fPIC -DP1HIP_KERNELS_CO='"$(CURDIR)/$(BUILD)/p1hip_kernels.hsaco"' -o $@ $<

$(BUILD)/p1hip_host.o: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $(CSRC)/p1hip.hip

p1_amd/libp1hip.so: $(BUILD)/p1hip_host.o $(BUILD)/p1hip_kernels_blob.o
	$(HIPCC) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# C++ host mirror of the reference's bitcoin package, LSP transport and the
# miner / server / client programs
HOSTSRC := p1_amd/host/bitcoin.cpp p1_amd/host/lsp_message.cpp p1_amd/host/lsp.cpp p1_amd/host/lspnet.cpp
HOSTHDR := p1_amd/host/bitcoin.hpp p1_amd/host/lsp_message.hpp p1_amd/host/gojson.hpp p1_amd/host/lsp.hpp \
           p1_amd/host/lspnet.hpp p1_amd/host/scheduler.hpp include/p1hip.h
HOSTFLAGS := -O2 -std=c++17 -Wall -Wextra -pthread

p1_amd/p1miner: p1_amd/host/p1miner.cpp p1_amd/host/miner_gpu.cpp $(HOSTSRC) $(HOSTHDR) p1_amd/libp1hip.so
	g++ $(HOSTFLAGS) -o $@ p1_amd/host/p1miner.cpp p1_amd/host/miner_gpu.cpp $(HOSTSRC) -Lp1_amd -lp1hip -Wl,-rpath,'$$ORIGIN'

# the server schedules; its pipe-transport miners are p1miner processes
p1_amd/p1server: p1_amd/host/p1server.cpp $(HOSTSRC) $(HOSTHDR)
	g++ $(HOSTFLAGS) -o $@ p1_amd/host/p1server.cpp $(HOSTSRC)

# the client never touches the GPU (client.go): no libp1hip link
p1_amd/p1client: p1_amd/host/p1client.cpp $(HOSTSRC) $(HOSTHDR)
	g++ $(HOSTFLAGS) -o $@ p1_amd/host/p1client.cpp $(HOSTSRC)

# test driver: the reference's LSP test scenarios (tests/test_lsp.py)
tools/lsp_scenarios: tests/lsp/lsp_scenarios.cpp p1_amd/host/lsp.cpp p1_amd/host/lspnet.cpp p1_amd/host/lsp_message.cpp $(HOSTHDR)
	g++ $(HOSTFLAGS) -o $@ tests/lsp/lsp_scenarios.cpp p1_amd/host/lsp.cpp p1_amd/host/lspnet.cpp p1_amd/host/lsp_message.cpp

# test double: an LSP miner answering with the CPU oracle (tests/test_lsp_bitcoin.py)
tools/lsp_fake_miner: tests/lsp/lsp_fake_miner.cpp p1_amd/host/bitcoin.cpp $(HOSTSRC) $(HOSTHDR) oracle
	g++ $(HOSTFLAGS) -o $@ tests/lsp/lsp_fake_miner.cpp $(HOSTSRC) -Loracle -lp1oracle -Wl,-rpath,'$$ORIGIN/../oracle'

# test program: hardware queues per process with and without a null-stream call
tools/queue_ctl: tools/queue_ctl.cpp include/p1hip.h p1_amd/libp1hip.so
	$(HIPCC) -O2 -std=c++17 -o $@ tools/queue_ctl.cpp -Lp1_amd -lp1hip -Wl,-rpath,'$$ORIGIN/../p1_amd'

# measurement program: WRITE_SIZE/FETCH_SIZE calibration for k_scan's partials
tools/wcal: tools/wcal.hip
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -o $@ tools/wcal.hip

# measurement library: shader-clock stamps around bench.py's timed steps
# (not linked into anything; bench.py loads it with ctypes)
tools/libp1clock.so: tools/clock_probe.hip
	$(HIPCC) -O2 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -Wall -o $@ tools/clock_probe.hip

# measurement program: XCD dispatch order, per-XCD clock and finish time under load
tools/xcd_probe: tools/xcd_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -o $@ tools/xcd_probe.hip

# measurement program: VALU issue cost vs operand VGPR banks
tools/vbank: tools/vbank.hip
	$(HIPCC) --offload-arch=gfx950 -O2 -std=c++17 -o $@ tools/vbank.hip

# host-only replay of the kernels' per-thread code (layout tests; not product)
tools/p1emu: tools/p1emu.cpp $(HDRS)
	$(HIPCC) -O2 -std=c++17 -DP1_NV2_PLAIN -o $@ tools/p1emu.cpp

oracle:
	$(MAKE) -C oracle

# Host code under sanitizers (tools/sanitize.sh, tests/test_sanitizers.py):
# ASan + UBSan (no recovery) and TSan builds of the LSP stack, the server
# scheduler, the client, the CPU test-double miner and the planner replay.
# ROCm's clang: its TSan intercepts pthread_cond_clockwait, which libstdc++
# uses for steady_clock waits and GCC 11's TSan does not (every condition
# wait then reads as a double lock).  p1emu includes the HIP headers, so it
# goes through hipcc with the sanitizers on the host side only.
SANCXX ?= /opt/rocm/lib/llvm/bin/clang++
SANBASE := -O1 -g -std=c++17 -pthread -fno-omit-frame-pointer
SAN_asan := -fsanitize=address,undefined -fno-sanitize-recover=undefined
SAN_tsan := -fsanitize=thread
SANDIR := $(BUILD)/san
SANPROGS := lsp_scenarios sched_test p1server p1client lsp_fake_miner
sanitize: $(foreach s,asan tsan,$(addprefix $(SANDIR)/$(s)/,$(SANPROGS)))
sanitize-emu: $(SANDIR)/asan/p1emu

$(SANDIR)/%/lsp_scenarios: tests/lsp/lsp_scenarios.cpp p1_amd/host/lsp.cpp p1_amd/host/lspnet.cpp p1_amd/host/lsp_message.cpp $(HOSTHDR)
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) $(SAN_$*) -o $@ tests/lsp/lsp_scenarios.cpp p1_amd/host/lsp.cpp p1_amd/host/lspnet.cpp p1_amd/host/lsp_message.cpp
$(SANDIR)/%/sched_test: tests/sched_test.cpp p1_amd/host/scheduler.hpp
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) $(SAN_$*) -o $@ tests/sched_test.cpp
$(SANDIR)/%/p1server: p1_amd/host/p1server.cpp $(HOSTSRC) $(HOSTHDR)
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) $(SAN_$*) -o $@ p1_amd/host/p1server.cpp $(HOSTSRC)
$(SANDIR)/%/p1client: p1_amd/host/p1client.cpp $(HOSTSRC) $(HOSTHDR)
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) $(SAN_$*) -o $@ p1_amd/host/p1client.cpp $(HOSTSRC)
$(SANDIR)/%/lsp_fake_miner: tests/lsp/lsp_fake_miner.cpp $(HOSTSRC) $(HOSTHDR) oracle
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) $(SAN_$*) -o $@ tests/lsp/lsp_fake_miner.cpp $(HOSTSRC) -L$(CURDIR)/oracle -lp1oracle -Wl,-rpath,$(CURDIR)/oracle
# the library's host runtime under ASan + UBSan (host side only: the kernels
# are the shipped code object) and its GPU stress driver; in tools/san, not
# build/, so that they travel to the GPU box with the tree
SANLIB := tools/san
sanitize-lib: $(SANLIB)/libp1hip.so $(SANLIB)/capi_san_stress $(SANLIB)/p1miner tools/asan_teardown
$(SANLIB)/p1miner: p1_amd/host/p1miner.cpp p1_amd/host/miner_gpu.cpp $(HOSTSRC) $(HOSTHDR) $(SANLIB)/libp1hip.so
	$(SANCXX) $(SANBASE) $(SAN_asan) -o $@ p1_amd/host/p1miner.cpp p1_amd/host/miner_gpu.cpp $(HOSTSRC) -L$(SANLIB) -lp1hip \
	    -Wl,-rpath,'$$ORIGIN'
$(SANLIB)/p1hip_host.o: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p $(@D)
	$(HIPCC) -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) -fno-omit-frame-pointer -Xarch_host -fsanitize=address \
	    -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -c -o $@ $(CSRC)/p1hip.hip
$(SANLIB)/libp1hip.so: $(SANLIB)/p1hip_host.o $(BUILD)/p1hip_kernels_blob.o
	$(HIPCC) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
$(SANLIB)/capi_san_stress: tests/capi_san_stress.cpp include/p1hip.h $(SANLIB)/libp1hip.so oracle
	$(SANCXX) $(SANBASE) $(SAN_asan) -Iinclude -o $@ tests/capi_san_stress.cpp -L$(SANLIB) -lp1hip \
	    -Wl,-rpath,'$$ORIGIN' -Loracle -lp1oracle -Wl,-rpath,'$$ORIGIN/../../oracle'

# measurement program: does ROCm's ASan runtime abort at exit without
# libp1hip at all (the r04p teardown CHECK)
tools/asan_teardown: tools/asan_teardown.cpp
	$(HIPCC) -O1 -g -std=c++17 -fno-omit-frame-pointer -Xarch_host -fsanitize=address -o $@ tools/asan_teardown.cpp \
	    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# the same under TSan (the device threads, barriers and the combine of a
# multi-device scan; the HIP runtime itself is not instrumented)
sanitize-lib-tsan: $(SANLIB)/tsan/libp1hip.so $(SANLIB)/tsan/capi_san_stress
$(SANLIB)/tsan/p1hip_host.o: $(CSRC)/p1hip.hip $(HDRS)
	mkdir -p $(@D)
	$(HIPCC) -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) -fno-omit-frame-pointer -Xarch_host -fsanitize=thread \
	    -c -o $@ $(CSRC)/p1hip.hip
$(SANLIB)/tsan/libp1hip.so: $(SANLIB)/tsan/p1hip_host.o $(BUILD)/p1hip_kernels_blob.o
	$(HIPCC) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
$(SANLIB)/tsan/capi_san_stress: tests/capi_san_stress.cpp include/p1hip.h $(SANLIB)/tsan/libp1hip.so oracle
	$(SANCXX) $(SANBASE) $(SAN_tsan) -Iinclude -o $@ tests/capi_san_stress.cpp -L$(SANLIB)/tsan -lp1hip \
	    -Wl,-rpath,'$$ORIGIN' -Loracle -lp1oracle -Wl,-rpath,'$$ORIGIN/../../../oracle'

$(SANDIR)/asan/p1emu: tools/p1emu.cpp $(HDRS)
	mkdir -p $(@D)
	$(HIPCC) -O1 -g -std=c++17 -fno-omit-frame-pointer -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -Xarch_host -fno-sanitize-recover=undefined -DP1_NV2_PLAIN -o $@ tools/p1emu.cpp

# libFuzzer harness of the wire codecs (tests/fuzz/fuzz_codecs.cpp) with
# ASan + UBSan.  -asan-globals=0: with -fsanitize=fuzzer this clang registers
# the harness's own string literals twice and ASan stops at start-up with a
# spurious odr-violation; heap, stack and UB checks are unaffected.
fuzz: $(SANDIR)/fuzz_codecs $(SANDIR)/fuzz_planner
# the host-side planner (make_plan, plan_shards); hipcc for the HIP headers,
# sanitizers and libFuzzer on the host side only
$(SANDIR)/fuzz_planner: tests/fuzz/fuzz_planner.cpp $(HDRS)
	mkdir -p $(@D)
	$(HIPCC) -O1 -g -std=c++17 -Xarch_host -fsanitize=fuzzer -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	    -Xarch_host -fno-sanitize-recover=undefined -o $@ tests/fuzz/fuzz_planner.cpp
$(SANDIR)/fuzz_codecs: tests/fuzz/fuzz_codecs.cpp p1_amd/host/bitcoin.cpp p1_amd/host/lsp_message.cpp $(HOSTHDR)
	mkdir -p $(@D)
	$(SANCXX) $(SANBASE) -fsanitize=fuzzer,address,undefined -fno-sanitize-recover=undefined -mllvm -asan-globals=0 \
	    -o $@ tests/fuzz/fuzz_codecs.cpp p1_amd/host/bitcoin.cpp p1_amd/host/lsp_message.cpp

# A/B tuning builds (not used unless P1HIP_LIB points at one):
#   make variant NAME=x DEVEXTRA='-DP1_FAST_WAVES=5' ISAPOST='--no-e64'
#   make variant NAME=nv2 DEVEXTRA=-DP1_NV2_PLAIN HOSTEXTRA=-DP1_NV2_PLAIN   (+ P1HIP_NO_SPLIT=1 at run time)
variant:
	$(MAKE) BUILD=build/var_$(NAME) DEVEXTRA="$(DEVEXTRA)" HIPFLAGS="$(HIPFLAGS) $(HOSTEXTRA)" ISAPOST="$(ISAPOST)" build/var_$(NAME)/p1hip_kernels_blob.o build/var_$(NAME)/p1hip_host.o
	mkdir -p p1_amd/variants
	$(HIPCC) -shared -fPIC -o p1_amd/variants/libp1hip_$(NAME).so build/var_$(NAME)/p1hip_host.o build/var_$(NAME)/p1hip_kernels_blob.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# ISA + resource report of the scan kernels (for DESIGN.md / profiling):
# build/p1hip_kernels.post.s is the exact assembly that ships
isa: $(BUILD)/p1hip_kernels.post.s
	$(HIPCC) $(DEVFLAGS) -c -o /dev/null $(CSRC)/p1hip_kernels.hip -Rpass-analysis=kernel-resource-usage 2> $(BUILD)/resource.txt || true

clean:
	rm -f p1_amd/libp1hip.so tools/libp1clock.so tools/queue_ctl tools/p1emu p1_amd/p1miner p1_amd/p1server p1_amd/p1client tools/lsp_scenarios tools/lsp_fake_miner tools/wcal tools/vbank
	rm -rf $(BUILD)/p1hip_kernels* $(BUILD)/p1hip_host.o
	$(MAKE) -C oracle clean
.PHONY: all oracle clean isa variant sanitize sanitize-emu sanitize-lib sanitize-lib-tsan fuzz
