# Build libislpose.so (HIP, gfx950) in-tree, and the oracle's reference build helpers.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := isl-signlanguage-translation_amd
CSRC     := $(PKG)/csrc
OUT      := $(PKG)/islpose/libislpose.so
# -ffp-contract=off: the post-processing kernels reproduce numpy/OpenCV fp32/fp64
# operation order bit-for-bit, which forbids fused multiply-adds.
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off -Iinclude -I$(CSRC) \
            -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-lambda-capture
SRCS     := $(CSRC)/conv.hip $(CSRC)/conv_x3.hip $(CSRC)/wino.hip $(CSRC)/wino_x3.hip $(CSRC)/ops.hip $(CSRC)/post.hip $(CSRC)/sign.hip $(CSRC)/runtime.cpp
OBJS     := $(patsubst $(CSRC)/%,build/%.o,$(SRCS))

all: $(OUT)

build/%.o: $(CSRC)/% $(CSRC)/internal.h include/islpose.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-z,defs -o $@ $(OBJS)

clean:
	rm -rf build $(OUT)

.PHONY: all clean

# development microbenchmark of the conv kernels (not part of the library)
tools/convbench: tools/convbench.cpp $(OBJS)
	$(HIPCC) $(HIPFLAGS) -x hip tools/convbench.cpp -x none $(filter-out build/runtime.cpp.o build/post.hip.o build/ops.hip.o,$(OBJS)) build/runtime.cpp.o build/post.hip.o build/ops.hip.o -o $@
