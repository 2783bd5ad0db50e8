# Builds the gfx950 kernel library behind the C ABI in include/vda.h.
#   make            -> video-depth-anything_amd/libvda.so (+ libvda_torch.so)
#   make tune       -> build/tune/libvda.so (+ libvda_torch.so): the same kernels with -DVDA_TUNING, which
#                      turns the route knobs into globals set through include/vda_tune.h (tests / tools only)
#   make oracle     -> nothing to compile (the oracle is a torch-CPU restatement), kept for symmetry
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := video-depth-anything_amd
SRCS    := $(wildcard $(PKG)/csrc/*.hip)
OBJS    := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRCS))
CXXFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -I include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form

all: $(PKG)/libvda.so $(PKG)/libvda_torch.so

# attention: no NaN inputs by construction, so max chains need no IEEE quieting (v_max3 straight
# off the MFMA results instead of canonicalising v_max per score); no SLP packing of the softmax sums
# into v_pk_add_f32 (slower beside MFMAs: spatial attention 303 -> 292 us without it)
build/vda_attn.o: EXTRA := -fno-honor-nans -mno-amdgpu-ieee -fno-slp-vectorize
# GEMM epilogues: SLP packing of scalar f32 math needs register moves that cost more than it saves
build/vda_gemm.o: EXTRA := -fno-slp-vectorize

build/tune/vda_attn.o: EXTRA := -fno-honor-nans -mno-amdgpu-ieee -fno-slp-vectorize
build/tune/vda_gemm.o: EXTRA := -fno-slp-vectorize
DEPS := $(PKG)/csrc/vda_common.h $(PKG)/csrc/vda_tune.h $(PKG)/csrc/phi_table.h include/vda.h include/vda_tune.h

build/%.o: $(PKG)/csrc/%.hip $(DEPS)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -c $< -o $@

build/tune/%.o: $(PKG)/csrc/%.hip $(DEPS)
	@mkdir -p build/tune
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -DVDA_TUNING -c $< -o $@

# -Bsymbolic: the library's internal calls bind to its own definitions, so the product and the tuning
# build can be loaded side by side in one process (the tests compare their routes)
$(PKG)/libvda.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,-Bsymbolic $(OBJS) -o $@

TUNE_OBJS := $(patsubst build/%,build/tune/%,$(OBJS))
build/tune/libvda.so: $(TUNE_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,-Bsymbolic $(TUNE_OBJS) -o $@

build/tune/libvda_torch.so: build/vda_torch.o build/tune/libvda.so
	$(CXX) build/vda_torch.o -o $@ $(subst -L $(PKG),-L build/tune,$(TORCH_LDFLAGS))

tune: build/tune/libvda.so build/tune/libvda_torch.so

# torch.ops.vda.* (TORCH_LIBRARY registration over the C ABI): host-only C++ against the installed
# PyTorch-ROCm headers, linked to libvda.so (found next to it through $$ORIGIN)
TORCH_DIR := $(shell python3 -c "import os, torch; print(os.path.dirname(torch.__file__))" 2>/dev/null)
TORCH_ABI := $(shell python3 -c "import torch; print(int(torch.compiled_with_cxx11_abi()))" 2>/dev/null)
TORCH_CXXFLAGS := -std=c++17 -O2 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$(TORCH_ABI) \
	-I include -I $(TORCH_DIR)/include -I $(TORCH_DIR)/include/torch/csrc/api/include -I /opt/rocm/include
TORCH_LDFLAGS := -shared -L $(TORCH_DIR)/lib -lc10 -lc10_hip -ltorch_cpu -ltorch_hip -ltorch \
	-L $(PKG) -lvda -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib

build/vda_torch.o: $(PKG)/csrc/vda_torch.cpp include/vda.h
	@mkdir -p build
	$(CXX) $(TORCH_CXXFLAGS) -c $< -o $@

$(PKG)/libvda_torch.so: build/vda_torch.o $(PKG)/libvda.so
	$(CXX) build/vda_torch.o -o $@ $(TORCH_LDFLAGS)

tools/mfma_probe: tools/mfma_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -Wno-unused-result $< -o $@

clean:
	rm -rf build $(PKG)/libvda.so $(PKG)/libvda_torch.so

.PHONY: all clean tune
