# Builds the HIP raster library for gfx950 in-tree (the .so travels to the GPU
# box with the snapshot) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG = libnativecpurenderer_amd
SRC = $(PKG)/csrc
OBJ ?= build/obj
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
           -fno-gpu-rdc -Wno-pass-failed -I$(SRC) $(EXTRA)
LIB ?= $(PKG)/libNativeCPURenderer.so
SRCS = $(wildcard $(SRC)/*.hip)
OBJS = $(patsubst $(SRC)/%.hip,$(OBJ)/%.o,$(SRCS))

all: $(LIB) oracle

$(OBJ)/%.o: $(SRC)/%.hip $(SRC)/nr_common.h $(SRC)/nr_tri.h $(SRC)/nr_tri_shade.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
