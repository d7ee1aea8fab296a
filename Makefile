# Native build: libthrs.so (HIP kernels for gfx950 + the C-ABI), the C++ test
# binary, and the CPU oracle.  Used by __graft_entry__.build().
#
# libthrs.so is linked from five translation units compiled in parallel: the
# C-ABI (thrs_capi.hip) and one launch-sequence unit per key type
# (thrs_run.hip with -DTHRS_RUN_KT=0..3).  Objects go to build/ (not shipped).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -fvisibility=hidden -Iinclude -Wall -Wno-unused-result -Wno-unused-function
PKG := tinyhipradixsort_amd
CSRC := $(PKG)/csrc
KSRC := $(CSRC)/thrs_host.hpp $(CSRC)/thrs_kernels.hpp $(CSRC)/thrs_hybrid.hpp $(CSRC)/thrs_fallback.hpp \
        include/thrs/thrs_capi.h
.DEFAULT_GOAL := all
KTS := 0 1 2 3

# one object set per build flavour: $(1) = directory, $(2) = extra flags
define objset
$(1)/capi.o: $(CSRC)/thrs_capi.hip $(KSRC)
	@mkdir -p $(1)
	$(HIPCC) $(HIPFLAGS) $(2) -c -o $$@ $$<
$(1)/run%.o: $(CSRC)/thrs_run.hip $(KSRC)
	@mkdir -p $(1)
	$(HIPCC) $(HIPFLAGS) $(2) -DTHRS_RUN_KT=$$* -c -o $$@ $$<
endef

OBJ := build/obj
OBJ_SPIN0 := build/obj_spin0
$(eval $(call objset,$(OBJ),))
# fault-injection build for the error-path tests only: every look-back /
# claim wait gives up at its first unpublished predecessor (THRS_SPIN_MAX=0),
# and thrs_debug_inject can make a plan's big-chunk list stale (THRS_FAULT_INJECT)
$(eval $(call objset,$(OBJ_SPIN0),-DTHRS_SPIN_MAX=0 -DTHRS_FAULT_INJECT))

all: $(PKG)/libthrs.so $(PKG)/libthrs_testutil.so $(PKG)/libthrs_vendor.so $(PKG)/libthrs_spin0.so \
     tests/cpp/unittest_thrs examples/helloworld oracle

$(PKG)/libthrs.so: $(OBJ)/capi.o $(foreach k,$(KTS),$(OBJ)/run$(k).o)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

$(PKG)/libthrs_spin0.so: $(OBJ_SPIN0)/capi.o $(foreach k,$(KTS),$(OBJ_SPIN0)/run$(k).o)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

$(PKG)/libthrs_testutil.so: $(CSRC)/thrs_testutil.hip $(CSRC)/thrs_kernels.hpp
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/thrs_testutil.hip

# vendor comparator (hipCUB/rocPRIM), benchmark-only
$(PKG)/libthrs_vendor.so: $(CSRC)/thrs_vendor.hip
	$(HIPCC) $(HIPFLAGS) -Wno-unused-parameter -shared -o $@ $<

CXX ?= g++
tests/cpp/unittest_thrs: tests/cpp/unittest_thrs.cpp include/thrs/tinyhipradixsort.hpp include/thrs/fpKey.hpp $(PKG)/libthrs.so
	$(CXX) -O2 -std=c++17 -fopenmp -Iinclude -o $@ $< -L$(PKG) -lthrs -Wl,-rpath,'$$ORIGIN/../../$(PKG)'

examples/helloworld: examples/helloworld.cpp include/thrs/tinyhipradixsort.hpp $(PKG)/libthrs.so
	$(CXX) -O2 -std=c++17 -Iinclude -o $@ $< -L$(PKG) -lthrs -Wl,-rpath,'$$ORIGIN/../$(PKG)'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(PKG)/*.so oracle/liboracle.so tests/cpp/unittest_thrs examples/helloworld
.PHONY: all clean oracle

# Tuning variants of libthrs.so for scripts/sweep.py / var_bench.sh:
#   make variants VARIANTS="name:-DFLAG=V+-DFLAG2=W ..." -j8
# -> exp/variants/libthrs_<name>.so
VARIANTS ?= stamps:-DTHRS_STAMPS
VNAMES := $(foreach v,$(VARIANTS),$(firstword $(subst :, ,$(v))))
vflags = $(subst +, ,$(word 2,$(subst :, ,$(filter $(1):%,$(VARIANTS)))))
$(foreach n,$(VNAMES),$(eval $(call objset,build/obj_v_$(n),$(call vflags,$(n)))))
exp/variants/libthrs_%.so: build/obj_v_%/capi.o $(foreach k,$(KTS),build/obj_v_%/run$(k).o)
	@mkdir -p exp/variants
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^
variants: $(foreach n,$(VNAMES),exp/variants/libthrs_$(n).so)
.PHONY: variants
