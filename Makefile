# Builds the in-tree C-ABI library dpdk_dc_sand_amd/libbf.so for gfx950 (MI355X) and the C oracle helpers.
# `python -c "import __graft_entry__ as g; g.build()"` drives this.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := dpdk_dc_sand_amd/csrc
LIB      := dpdk_dc_sand_amd/libbf.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics
SRCS     := $(CSRC)/bf_runtime.cpp $(CSRC)/bf_coeff.hip $(CSRC)/bf_reorder.hip $(CSRC)/bf_beamform.hip \
            $(CSRC)/bf_fused.hip $(CSRC)/bf_wide.hip $(CSRC)/bf_wide_i8.hip $(CSRC)/bf_q14table.hip $(CSRC)/bf_requant.hip \
            $(CSRC)/bf_study.hip $(CSRC)/bf_pipeline.cpp $(CSRC)/bf_comm.cpp
OBJS     := $(patsubst $(CSRC)/%,build/%.o,$(SRCS))
HDRS     := $(wildcard $(CSRC)/*.hpp) $(wildcard $(CSRC)/diag/*.inc) include/bf.h

.PHONY: all clean diag cabi stream
all: $(LIB) cabi

# bench.py's stream ceiling (the box's best plain stream over a kernel's byte mix): a small library of its own, so the
# GPU box needs no diagnostic build.
STREAM_LIB := build/libbf_stream.so
stream: $(STREAM_LIB)
$(STREAM_LIB): tools/stream_ceiling.hip $(CSRC)/diag/stream_kernels.hpp
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# C callers of the ABI (tests/test_c_abi.py): the harness-order smoke and INTEGRATION.md's streaming example,
# compiled from the markdown block itself.  Plain C against include/bf.h, linked to the in-tree libbf.so.
CC       ?= gcc
CABI     := build/bf_smoke build/bf_stream_doc
cabi: $(CABI)
build/stream_snippet.inc: INTEGRATION.md
	@mkdir -p build
	awk '/<!-- snippet: stream -->/{f=1; next} f && /^```c/{p=1; next} p && /^```/{exit} p' $< > $@
	@test -s $@ || { echo "no stream snippet in INTEGRATION.md"; rm -f $@; exit 1; }
build/bf_smoke: tests/c/bf_smoke.c include/bf.h $(LIB)
	@mkdir -p build
	$(CC) -std=c11 -O2 -Wall -Iinclude $< -o $@ -L$(dir $(LIB)) -lbf -lm -Wl,-rpath,'$$ORIGIN/../$(dir $(LIB))'
build/bf_stream_doc: tests/c/bf_stream_doc.c build/stream_snippet.inc include/bf.h $(LIB)
	@mkdir -p build
	$(CC) -std=c11 -O2 -Wall -Iinclude -Ibuild $< -o $@ -L$(dir $(LIB)) -lbf -Wl,-rpath,'$$ORIGIN/../$(dir $(LIB))'

build/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

clean:
	rm -rf build $(LIB)

# Diagnostic build (ablation variants + HBM stream kernel); used only by tools/diag_*.py and bench.py's stream
# ceiling, never by the product.  The measured-slower kernels and the measurement entry points live in
# $(CSRC)/diag/ (*.inc included under -DBF_DIAG, and the diagnostic-only bf_wide_i8os.hip).
DIAG_LIB := build/libbf_diag.so
DIAG_SRCS := $(SRCS) $(CSRC)/diag/bf_wide_i8os.hip
DIAG_OBJS := $(patsubst $(CSRC)/%,build/diag/%.o,$(DIAG_SRCS))
diag: $(DIAG_LIB)
build/diag/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DBF_DIAG -x hip -c $< -o $@
$(DIAG_LIB): $(DIAG_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(DIAG_OBJS) -ldl
