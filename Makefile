# Build recipe for the MI355X ray tracer (no cmake): `make -j8` (what __graft_entry__.build() runs).
#   parallel-ray-tracer_amd/lib/librt_host.so   host half: loader, camera, BVH, BMP (g++, strict FP)
#   parallel-ray-tracer_amd/lib/librt_hip.so    device half: HIP kernels for gfx950 + the rt_* C-ABI (RCCL dlopen'ed on first use)
#   parallel-ray-tracer_amd/bin/raytracer       CLI drop-in for cpu/raytracer (links both)
#   oracle/liboracle*.so, oracle/_ref/*         test infrastructure (oracle/Makefile)
PKG      := parallel-ray-tracer_amd
CSRC     := $(PKG)/csrc
LIB      := $(PKG)/lib
BIN      := $(PKG)/bin
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950

# Strict IEEE fp32 everywhere on the parity path: no contraction, no fast-math, IEEE div/sqrt.
# -fno-slp-vectorize: the SLP vectoriser packed the triangle tests and shading into v_pk_{mul,add}_f32 pairs whose
# operand shuffles cost as many moves as they saved, and its register pairs pushed the walks to the 128-VGPR cap
# (same box: dragon 0.519 -> 0.511 ms per frame, car_boxed 0.746 -> 0.697, sportscar 0.787 -> 0.757).
HOST_FLAGS := -O2 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -pthread -Wall -Wextra -Iinclude
HIP_FLAGS  := -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -fno-slp-vectorize $(PRT_DEFS) \
              -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -Wall -Iinclude -I$(CSRC)

.PHONY: all host hip cli oracle clean asan

all: host hip cli oracle

host: $(LIB)/librt_host.so
hip: $(LIB)/librt_hip.so
cli: $(BIN)/raytracer

HOST_SRCS := $(CSRC)/host/rt_host.cpp $(CSRC)/host/rt_wide.cpp $(CSRC)/host/rt_cache.cpp

$(LIB)/librt_host.so: $(HOST_SRCS) include/rt_host.h include/rt_types.h
	@mkdir -p $(LIB)
	g++ $(HOST_FLAGS) -shared -o $@ $(HOST_SRCS)

HIP_SRCS := $(CSRC)/hip/rt_hip.hip
HIP_HDRS := $(wildcard $(CSRC)/hip/*.hpp) include/rt_hip.h include/rt_types.h

$(LIB)/librt_hip.so: $(HIP_SRCS) $(HIP_HDRS) $(LIB)/librt_host.so
	@mkdir -p $(LIB)
	$(HIPCC) $(HIP_FLAGS) -shared -o $@ $(HIP_SRCS) -L$(LIB) -lrt_host -ldl -Wl,-rpath,'$$ORIGIN'


$(BIN)/raytracer: $(CSRC)/cli/raytracer.cpp $(LIB)/librt_host.so $(LIB)/librt_hip.so
	@mkdir -p $(BIN)
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude -o $@ $(CSRC)/cli/raytracer.cpp \
	    -L$(LIB) -lrt_host -lrt_hip -Wl,-rpath,'$$ORIGIN/../lib' -pthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(LIB) $(BIN)
	$(MAKE) -C oracle clean

# exhaustive check of rtd::rcp_ieee against IEEE division (test infrastructure, tests/test_gpu_rcp.py)
RCP_CHECK := tools/rcp/rcp_exhaustive
hip: $(RCP_CHECK)
$(RCP_CHECK): tools/rcp/rcp_exhaustive.hip $(CSRC)/hip/rt_device.hpp
	$(HIPCC) $(HIP_FLAGS) -o $@ $<

# Sanitizer build of the host library (SURVEY §5 "race detection / sanitizers"): librt_host.so -- the OBJ/MTL parser
# restating cpu/src/triangle.c:26-126, the BVH builders, the wide collapse (rt_wide.cpp), the scene cache -- with
# AddressSanitizer + UndefinedBehaviorSanitizer (any report is fatal), then the host-side tests against it
# (prt._lib loads it through PRT_LIB_DIR; libasan is preloaded ahead of whatever LD_PRELOAD already holds, as ASan
# must come first). Build container only (CPU; no GPU code is involved).
ASAN_DIR   := build/asan
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all
$(ASAN_DIR)/librt_host.so: $(HOST_SRCS) include/rt_host.h include/rt_types.h
	@mkdir -p $(ASAN_DIR)
	g++ $(HOST_FLAGS) $(ASAN_FLAGS) -shared -o $@ $(HOST_SRCS)

asan: $(ASAN_DIR)/librt_host.so oracle
	PRT_LIB_DIR=$(CURDIR)/$(ASAN_DIR) ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
	UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	LD_PRELOAD="$$(g++ -print-file-name=libasan.so)$${LD_PRELOAD:+:$$LD_PRELOAD}" \
	python3 -m pytest -q -m "not gpu" -p no:cacheprovider tests/test_host.py tests/test_oracle.py
