# Build of the MI355X (gfx950) SIFT path.  Outputs stay in-tree so they
# travel to the GPU box with the snapshot (they are git-ignored).
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := sift-scale-space-extrema-detection_amd
CSRC    := $(PKG)/csrc
HIPSRC  := $(CSRC)/sift_gauss.hip $(CSRC)/sift_extrema.hip $(CSRC)/sift_refine.hip $(CSRC)/sift_image.hip $(CSRC)/sift_api.hip
HDRS    := $(wildcard $(CSRC)/*.h) include/sift_hip.h
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result
LIB     := $(PKG)/libsift_hip.so
OBJS    := $(patsubst $(CSRC)/%.hip,$(PKG)/build/%.o,$(HIPSRC))

all: lib oracle
lib: $(LIB)

$(PKG)/build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(PKG)/build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(PKG)/build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean
