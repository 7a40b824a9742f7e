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
HOST_FLAGS := -O2 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -Wall -Wextra -Iinclude
HIP_FLAGS  := -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math $(PRT_DEFS) \
              -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -Wall -Iinclude -I$(CSRC)

.PHONY: all host hip cli oracle clean

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
