# Build the MI355X (gfx950) shared library and the oracle's C pieces.
#   make            -> interiorpoint-gpu_amd/ipm355/libipm355.so
#   make clean
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
SRC_DIR  := interiorpoint-gpu_amd/csrc
OUT      := interiorpoint-gpu_amd/ipm355/libipm355.so
OBJ_DIR  := build/obj
# -ffp-contract=off: elementwise arithmetic rounds like NumPy (separate multiply / add);
# dot products and MFMA use explicit fma where intended.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
            -Wno-unused-variable -Wno-unused-result -Wno-unused-value -Iinclude -I$(SRC_DIR)
SRCS     := $(SRC_DIR)/ipm_blas.hip $(SRC_DIR)/ipm_barrier.hip $(SRC_DIR)/ipm_engine.hip
OBJS     := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
HDRS     := $(SRC_DIR)/ipm_common.h $(SRC_DIR)/ipm_mfma.h $(SRC_DIR)/ipm_barrier.h include/ipm355.h

all: $(OUT)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -rf build $(OUT)

.PHONY: all clean
