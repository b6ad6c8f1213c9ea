# libsfmcore.so: hand-written HIP for gfx950 + host C++ (C-ABI in include/sfmcore.h)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := 3dreconstruction_amd
CSRC := $(PKG)/csrc
LIB := $(PKG)/lib/libsfmcore.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -mcode-object-version=5 \
            -Wall -Wno-unused-result -I/opt/rocm/include
SRCS := $(wildcard $(CSRC)/*.cpp $(CSRC)/*.hip)
OBJS := $(patsubst $(CSRC)/%,build/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.h) include/sfmcore.h $(wildcard $(PKG)/include/sfm/*.hpp)

all: $(LIB) oracle/liboracle.so tests/cpp/facade_test tests/cpp/plan_pool_test

build/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -fvisibility=hidden -fvisibility-inlines-hidden -x hip -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(PKG)/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

oracle/liboracle.so: FORCE
	$(MAKE) -C oracle

FORCE:

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all clean FORCE

# C++ façade test (links the product and, as the checker, the oracle)
tests/cpp/facade_test: tests/cpp/facade_test.cpp 3dreconstruction_amd/include/sfm/sfm.hpp 3dreconstruction_amd/include/sfm/world.hpp $(LIB) oracle/liboracle.so
	g++ -O2 -std=c++17 -Wall -o $@ $< -I/opt/rocm/include -L3dreconstruction_amd/lib -Loracle -lsfmcore -loracle \
	    -Wl,-rpath,'$$ORIGIN/../../3dreconstruction_amd/lib' -Wl,-rpath,'$$ORIGIN/../../oracle'

# planner worker-pool stress test (host only, no GPU)
tests/cpp/plan_pool_test: tests/cpp/plan_pool_test.cpp $(CSRC)/ba_plan.cpp $(HDRS)
	g++ -O2 -std=c++17 -w -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< -L/opt/rocm/lib -lamdhip64 -lpthread \
	    -Wl,-rpath,/opt/rocm/lib
