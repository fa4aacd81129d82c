# Build the MI355X (gfx950) shared library libipm355.so (the oracle is pure Python: nothing to build).
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
SRCS     := $(SRC_DIR)/ipm_blas.hip $(SRC_DIR)/ipm_barrier.hip $(SRC_DIR)/ipm_engine.hip $(SRC_DIR)/ipm_lasso.hip $(SRC_DIR)/ipm_lstsq.hip
# no vendor math libraries: every kernel is hand-written (the least-squares fallback's
# eigensolver included, ipm_lstsq.hip)
LIBS     :=
OBJS     := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
HDRS     := $(SRC_DIR)/ipm_common.h $(SRC_DIR)/ipm_mfma.h $(SRC_DIR)/ipm_barrier.h $(SRC_DIR)/ipm_handle.h include/ipm355.h

all: $(OUT)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@ $(LIBS)

# diagnostic library: per-workgroup role timestamps of one Cholesky launch (IPM_TRACE_BLOCK=b),
# loaded with IPM355_LIB=build/trace/libipm355_trace.so (scripts/role_trace.py)
TRACE_OUT := build/trace/libipm355_trace.so
trace: $(TRACE_OUT)
$(TRACE_OUT): $(SRCS) $(HDRS)
	@mkdir -p build/trace
	$(HIPCC) $(HIPFLAGS) -DIPM_ROLE_TRACE -c $(SRC_DIR)/ipm_blas.hip -o build/trace/ipm_blas.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC build/trace/ipm_blas.o $(OBJ_DIR)/ipm_barrier.o \
	    $(OBJ_DIR)/ipm_engine.o $(OBJ_DIR)/ipm_lasso.o $(OBJ_DIR)/ipm_lstsq.o -o $@ $(LIBS)

clean:
	rm -rf build $(OUT)

.PHONY: all clean trace
