# Builds the in-tree C-ABI library dpdk_dc_sand_amd/libbf.so for gfx950 (MI355X) and the C oracle helpers.
# `python -c "import __graft_entry__ as g; g.build()"` drives this.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := dpdk_dc_sand_amd/csrc
LIB      := dpdk_dc_sand_amd/libbf.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics
SRCS     := $(CSRC)/bf_runtime.cpp $(CSRC)/bf_coeff.hip $(CSRC)/bf_reorder.hip $(CSRC)/bf_beamform.hip \
            $(CSRC)/bf_fused.hip $(CSRC)/bf_wide.hip $(CSRC)/bf_wide_i8.hip $(CSRC)/bf_requant.hip \
            $(CSRC)/bf_pipeline.cpp
OBJS     := $(patsubst $(CSRC)/%,build/%.o,$(SRCS))
HDRS     := $(wildcard $(CSRC)/*.hpp) include/bf.h

.PHONY: all clean diag
all: $(LIB)

build/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(LIB)

# Diagnostic build (ablation variants + HBM stream kernel); used only by tools/diag_*.py, never by the product.
DIAG_LIB := build/libbf_diag.so
diag: $(DIAG_LIB)
$(DIAG_LIB): $(SRCS) $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DBF_DIAG -shared -o $@ $(SRCS)
