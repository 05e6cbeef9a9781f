# Builds libhohgpu.so (all HIP kernels for gfx950 + host orchestration) in-tree, the C++ CLIs
# (choh / dhoh drop-ins) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := hoh-ans_amd/csrc
LIBDIR := hoh-ans_amd/lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result
# make DEBUG_READ=1: export hoh_debug_read (tools/scripts/*_dbg.py); never in the product build
ifeq ($(DEBUG_READ),1)
HIPFLAGS += -DHOH_DEBUG_READ
endif
SRCS := $(wildcard $(CSRC)/*.hip) $(wildcard $(CSRC)/*.cpp)
OBJS := $(patsubst $(CSRC)/%,build/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.h) include/hoh_ans.h

BINDIR := hoh-ans_amd/bin

all: $(LIBDIR)/libhohgpu.so oracle/liboracle.so $(BINDIR)/choh $(BINDIR)/dhoh $(BINDIR)/dropin_test

build/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libhohgpu.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl -lpthread

$(BINDIR)/%: tools/cli/%.cpp tools/cli/gpus.h $(LIBDIR)/libhohgpu.so include/hoh_ans.h $(wildcard include/hoh/*.hpp)
	@mkdir -p $(BINDIR)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -o $@ $< -L$(LIBDIR) -lhohgpu -Wl,-rpath,'$$ORIGIN/../lib'

oracle/liboracle.so: oracle/hoh_oracle.c oracle/hoh_oracle.h
	gcc -O2 -shared -fPIC -o $@ oracle/hoh_oracle.c -lm

clean:
	rm -rf build $(LIBDIR)/libhohgpu.so oracle/liboracle.so $(BINDIR)

.PHONY: all clean
