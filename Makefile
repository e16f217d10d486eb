# Build of the MI355X classifier (gfx950) and of the CPU oracle.
#   make            -> ingress-node-firewall_amd/lib/libinfw.so          (product: C ABI + HIP kernels)
#                      ingress-node-firewall_amd/lib/libinfw_workload.so (bench/test workload generator)
#                      oracle/build/liborc.so                            (test-only CPU oracle)
#                      ingress-node-firewall_amd/lib/libinfw_loader.so   (host side: C++ pkg/ebpf + pkg/metrics)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CC       ?= gcc
PKG      := ingress-node-firewall_amd
SRC      := $(PKG)/csrc
OUT      := $(PKG)/lib
OBJ      := $(PKG)/build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -Iinclude
EXTRA    ?=

LIB_SRCS := $(SRC)/abi.cpp $(SRC)/image.cpp $(SRC)/tables.cpp $(SRC)/incremental.cpp $(SRC)/controlplane.cpp \
            $(SRC)/hostfeed.cpp $(SRC)/classify.hip $(SRC)/pack.hip $(SRC)/patch.hip
LIB_OBJS := $(patsubst $(SRC)/%,$(OBJ)/%.o,$(LIB_SRCS))
HDRS     := include/infw.h include/infw_host.h $(wildcard $(SRC)/*.h)

all: $(OUT)/libinfw.so $(OUT)/libinfw_workload.so oracle/build/liborc.so $(OUT)/libinfw_loader.so $(OUT)/infw_loader_test

# classify.hip: the LDS counter atomics are issued by one lane or at per-lane addresses, where the atomic
# optimizer's wave scan (mbcnt, ballot count, multiply) is pure overhead in the hot loop
$(OBJ)/classify.hip.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None

# build id (infw_build_id()): a hash of the kernel / table-layout sources and the flags they are compiled with;
# bench.py only attaches a profile's PMC figures to a line when the profile was taken on the same build id
# (and a table image is accepted only by a library of the same build id, so every source that defines the serialised
# layout — image.cpp's field order, infw_internal.h's HostTables / IncState, incremental.cpp's state — is in it)
BUILDID_SRCS := $(SRC)/classify.hip $(SRC)/infw_tables.h $(SRC)/infw_launch.h $(SRC)/infw_pack.h $(SRC)/infw_hostpack.h $(SRC)/tables.cpp $(SRC)/pack.hip include/infw.h \
                $(SRC)/image.cpp $(SRC)/infw_internal.h $(SRC)/incremental.cpp
# The flags part is fixed when the Makefile is read (abi.cpp's, which compiles the id in): a target-specific HIPFLAGS
# of whichever target first needs the header (classify.hip.o's, abi.cpp.o's, the sanitizer objects') must not change it.
BUILDID_FLAGS := $(HIPFLAGS) -I$(OBJ)
$(OBJ)/infw_build_id.h: $(BUILDID_SRCS) Makefile
	@mkdir -p $(OBJ)
	@printf '#define INFW_BUILD_ID "%s"\n' "$$( (cat $(BUILDID_SRCS); echo '$(BUILDID_FLAGS) $(EXTRA) $(ARCH)') | sha256sum | cut -c1-16)" > $@.tmp
	@cmp -s $@.tmp $@ && rm -f $@.tmp || mv $@.tmp $@
$(OBJ)/abi.cpp.o: $(OBJ)/infw_build_id.h
$(OBJ)/abi.cpp.o: HIPFLAGS += -I$(OBJ)

$(OBJ)/%.o: $(SRC)/% $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $< -o $@

$(OUT)/libinfw.so: $(LIB_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $@ $(LIB_OBJS)

$(OUT)/libinfw_workload.so: $(OBJ)/workload.hip.o
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $<

# host side above the C ABI: the C++ form of pkg/ebpf IngNodeFwController + pkg/metrics (the reference's host
# side is Go, absent here), and the driver tests/test_loader_cpp.py runs it through
HOST := $(PKG)/host
$(OUT)/libinfw_loader.so: $(HOST)/infw_loader.cpp $(HOST)/infw_loader.hpp include/infw.h $(OUT)/libinfw.so
	$(CXX) -std=c++17 -O2 -fPIC -shared -Wall -Wextra -o $@ $(HOST)/infw_loader.cpp -L$(OUT) -linfw -Wl,-rpath,'$$ORIGIN'
# (in lib/, beside the libraries, so the GPU box gets the binary with them: tests/test_loader_cpp.py runs it there too)
$(OUT)/infw_loader_test: tests/c/loader_test.cpp $(OUT)/libinfw_loader.so
	$(CXX) -std=c++17 -O2 -Wall -Wextra -o $@ tests/c/loader_test.cpp -L$(OUT) -linfw_loader -linfw -Wl,-rpath,'$$ORIGIN'

oracle/build/liborc.so: oracle/infw_oracle.c oracle/infw_oracle.h
	@mkdir -p oracle/build
	$(CC) -O2 -g -fPIC -shared -pthread -Wall -Wextra -o $@ oracle/infw_oracle.c

# kernel resource usage (VGPR/SGPR/LDS/occupancy) of the classify kernels
resource-usage:
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-atomic-optimizer-strategy=None -Rpass-analysis=kernel-resource-usage -c $(SRC)/classify.hip -o /tmp/classify_ru.o

asm:
	@mkdir -p $(OBJ)/asm
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-atomic-optimizer-strategy=None --offload-device-only -S -o $(OBJ)/asm/classify.s $(SRC)/classify.hip

# host-only sanitizer run of the table compiler + shared walk (no GPU code involved)
asan:
	@mkdir -p $(OBJ)
	g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=undefined -Iinclude \
	    tools/asan_walk.cpp $(SRC)/tables.cpp $(SRC)/incremental.cpp $(SRC)/controlplane.cpp -o $(OBJ)/asan_walk
	$(OBJ)/asan_walk

# AddressSanitizer/UBSan builds of the whole host side (CPU only; the gfx950 kernels' objects are the product's, their
# device code is not instrumented): libinfw.so's host sources, the C++ loader and its driver, and tools/asan_abi.cpp,
# which drives the host-only paths of the C ABI (map edits, commits, key walks, debug walk, encoders, table image
# export / import incl. corrupt images).  tests/test_compiler_cpu.py and tests/test_loader_cpp.py run them.
ASAN_DIR   := $(OBJ)/asan
ASAN_FLAGS := -std=c++17 -g -O1 -fPIC -fsanitize=address,undefined -fno-sanitize-recover=undefined \
              -fno-omit-frame-pointer -Iinclude -I$(OBJ) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
ASAN_SRCS  := $(SRC)/abi.cpp $(SRC)/image.cpp $(SRC)/tables.cpp $(SRC)/incremental.cpp $(SRC)/controlplane.cpp \
              $(SRC)/hostfeed.cpp
ASAN_OBJS  := $(patsubst $(SRC)/%,$(ASAN_DIR)/%.o,$(ASAN_SRCS))
HIP_OBJS   := $(OBJ)/classify.hip.o $(OBJ)/pack.hip.o $(OBJ)/patch.hip.o
$(ASAN_DIR)/%.o: $(SRC)/% $(HDRS) $(OBJ)/infw_build_id.h
	@mkdir -p $(ASAN_DIR)
	g++ $(ASAN_FLAGS) -c $< -o $@
$(ASAN_DIR)/libinfw.so: $(ASAN_OBJS) $(HIP_OBJS)
	g++ -shared -fsanitize=address,undefined -o $@ $^ -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
$(ASAN_DIR)/libinfw_loader.so: $(HOST)/infw_loader.cpp $(HOST)/infw_loader.hpp $(ASAN_DIR)/libinfw.so
	g++ $(ASAN_FLAGS) -shared -o $@ $(HOST)/infw_loader.cpp -L$(ASAN_DIR) -linfw -Wl,-rpath,'$$ORIGIN'
$(ASAN_DIR)/infw_loader_test: tests/c/loader_test.cpp $(ASAN_DIR)/libinfw_loader.so
	g++ $(ASAN_FLAGS) -o $@ tests/c/loader_test.cpp -L$(ASAN_DIR) -linfw_loader -linfw -Wl,-rpath,'$$ORIGIN'
$(ASAN_DIR)/asan_abi: tools/asan_abi.cpp $(ASAN_DIR)/libinfw.so
	g++ $(ASAN_FLAGS) -o $@ tools/asan_abi.cpp -L$(ASAN_DIR) -linfw -Wl,-rpath,'$$ORIGIN'
asan-host: $(ASAN_DIR)/asan_abi $(ASAN_DIR)/infw_loader_test

# ThreadSanitizer build of the same host sources and tools/tsan_abi.cpp, which runs the C ABI's threading contract
# (include/infw.h "threads": a control-plane thread committing epochs while reader threads walk, read and introspect)
# on a host-only context.  tests/test_threads_cpu.py runs it.
TSAN_DIR   := $(OBJ)/tsan
TSAN_FLAGS := -std=c++17 -g -O1 -fPIC -fsanitize=thread -fno-omit-frame-pointer -Iinclude -I$(OBJ) -I/opt/rocm/include \
              -D__HIP_PLATFORM_AMD__
TSAN_OBJS  := $(patsubst $(SRC)/%,$(TSAN_DIR)/%.o,$(ASAN_SRCS))
$(TSAN_DIR)/%.o: $(SRC)/% $(HDRS) $(OBJ)/infw_build_id.h
	@mkdir -p $(TSAN_DIR)
	g++ $(TSAN_FLAGS) -c $< -o $@
$(TSAN_DIR)/libinfw.so: $(TSAN_OBJS) $(HIP_OBJS)
	g++ -shared -fsanitize=thread -o $@ $^ -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
$(TSAN_DIR)/tsan_abi: tools/tsan_abi.cpp $(TSAN_DIR)/libinfw.so
	g++ $(TSAN_FLAGS) -o $@ tools/tsan_abi.cpp -L$(TSAN_DIR) -linfw -Wl,-rpath,'$$ORIGIN'
# the packer pool of infw_classify_xdp_host alone (no device), its coordinator played by the test
$(TSAN_DIR)/tsan_hostpool: tools/tsan_hostpool.cpp $(TSAN_DIR)/hostfeed.cpp.o
	g++ $(TSAN_FLAGS) -pthread -o $@ tools/tsan_hostpool.cpp $(TSAN_DIR)/hostfeed.cpp.o
tsan-host: $(TSAN_DIR)/tsan_abi $(TSAN_DIR)/tsan_hostpool

clean:
	rm -rf $(OBJ) $(OUT) oracle/build

.PHONY: all clean resource-usage asm asan asan-host tsan-host cachesim patch_bench

# host model of the L2 behaviour of the table walk (layout experiments; tools/cachesim.cpp)
cachesim: $(OUT)/libinfw_workload.so
	@mkdir -p $(OBJ)
	g++ -std=c++17 -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/cachesim.cpp $(SRC)/tables.cpp \
	    $(SRC)/incremental.cpp $(SRC)/controlplane.cpp -L$(OUT) -linfw_workload -Wl,-rpath,$(abspath $(OUT)) \
	    -o $(OBJ)/cachesim

# host cost of incremental commits per phase (tools/patch_bench.cpp)
patch_bench: $(OUT)/libinfw_workload.so
	@mkdir -p $(OBJ)
	g++ -std=c++17 -O3 -pthread -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/patch_bench.cpp \
	    $(SRC)/tables.cpp $(SRC)/incremental.cpp $(SRC)/controlplane.cpp $(SRC)/image.cpp -L$(OUT) -linfw_workload \
	    -Wl,-rpath,$(abspath $(OUT)) -o $(OBJ)/patch_bench
