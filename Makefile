# Build of libhuygens_hip.so (gfx950 only) and the CPU oracle.
#   make            -> huygens_amd/lib/libhuygens_hip.so + oracle/_build/libhz_oracle.so
#   make -j8 lib    -> the HIP library only
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function \
            -Wno-pass-failed -munsafe-fp-atomics
LDFLAGS ?= -shared
LIBDIR := huygens_amd/lib
OBJDIR := build/obj
SRCS := $(wildcard huygens_amd/csrc/*.hip)
OBJS := $(patsubst huygens_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRCS))
HDRS := $(wildcard huygens_amd/csrc/*.h) include/huygens_hip.h

all: lib oracle

lib: $(LIBDIR)/libhuygens_hip.so

$(OBJDIR)/%.o: huygens_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -c $< -o $@

# per-file flags: the correction GEMM keeps its MFMA accumulators in VGPRs (no AGPR copies
# around the k loop)
HIPFLAGS_hz_fb_gemm := -mllvm -amdgpu-mfma-vgpr-form=1

$(LIBDIR)/libhuygens_hip.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(LDFLAGS) -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIBDIR)/*.so
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean
