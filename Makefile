# Build of the MI355X path-tracing hot path.
#   librtpt.so   gfx950 HIP kernel + C-ABI (include/rtpt.h)     -> gpuraytracer_amd/
#   rtrace       C++ CLI host (mirrors RTrace/main.swift)       -> gpuraytracer_amd/
#   oracle       CPU oracle for tests / cpu_baseline            -> oracle/liboracle.so
# Every TU is compiled with -ffp-contract=off: the arithmetic contract of
# DESIGN.md §3 (explicit fmaf only) that makes GPU == oracle bit-exact.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := gpuraytracer_amd
SRC := $(PKG)/csrc
BLD ?= build
COMMON := -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude
HOSTCXX ?= /opt/rocm/llvm/bin/clang++
HIPFLAGS := $(COMMON) --offload-arch=$(ARCH) -fno-slp-vectorize $(EXTRA)
HOSTFLAGS := $(COMMON) -D__HIP_PLATFORM_AMD__ -isystem /opt/rocm/include $(EXTRA)

OBJS := $(BLD)/rt_kernel.o $(BLD)/rt_mis.o $(BLD)/rt_lbvh.o $(BLD)/rt_gsah.o $(BLD)/rt_api.o $(BLD)/rt_scene.o $(BLD)/rt_image.o
HDRS := include/rtpt.h include/rt_types.h $(SRC)/rt_math.h $(SRC)/rt_kernel.hpp $(SRC)/rt_scene.hpp $(SRC)/rt_halton.hpp

LIB ?= $(PKG)/librtpt.so
# Hash of every source the library is built from (gpuraytracer_amd/srchash.py),
# compiled into rt_api.o as rt_build_sha(): the loader refuses a stale binary.
ALLSRC := $(wildcard $(SRC)/*.hip $(SRC)/*.hpp $(SRC)/*.h $(SRC)/*.cpp include/*.h)
SRC_SHA := $(shell python3 $(PKG)/srchash.py)

all: $(LIB) $(PKG)/rtrace oracle

lib: $(LIB)

$(BLD):
	mkdir -p $(BLD)

$(BLD)/%.o: $(SRC)/%.hip $(HDRS) $(SRC)/rt_trace.hpp | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BLD)/rt_api.o: $(SRC)/rt_api.cpp $(ALLSRC) | $(BLD)
	$(HOSTCXX) $(HOSTFLAGS) -DRT_SRC_SHA='"$(SRC_SHA)"' -c $< -o $@

$(BLD)/%.o: $(SRC)/%.cpp $(HDRS) | $(BLD)
	$(HOSTCXX) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,--no-undefined

$(PKG)/rtrace: $(SRC)/rtrace_main.cpp $(PKG)/librtpt.so $(HDRS)
	$(HOSTCXX) $(HOSTFLAGS) -o $@ $< -L$(PKG) -lrtpt -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

# ---- sanitizer build of the CPU code (ASan/UBSan) -------------------
# build_asan/liboracle.so  the oracle, -fsanitize=address,undefined
# build_asan/librtpt.so    the host C++ of the library (scene compile, host BVH
#                          builds on host threads, tile layout/placement, image
#                          epilogue, C-ABI argument handling) sanitized, linked
#                          with the device objects of build/
# `make asan-test` runs the CPU tests of that code (tests/run_sanitized.py)
# under it; UBSan findings abort (-fno-sanitize-recover).
ASAN := build_asan
SAN := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -shared-libasan
ASAN_RT := $(shell $(HOSTCXX) -print-file-name=libclang_rt.asan-x86_64.so)
ASAN_HOST := $(ASAN)/rt_api.o $(ASAN)/rt_scene.o $(ASAN)/rt_image.o

$(ASAN):
	mkdir -p $(ASAN)

$(ASAN)/rt_api.o: $(SRC)/rt_api.cpp $(ALLSRC) | $(ASAN)
	$(HOSTCXX) $(HOSTFLAGS) $(SAN) -DRT_SRC_SHA='"$(SRC_SHA)"' -c $< -o $@

$(ASAN)/%.o: $(SRC)/%.cpp $(HDRS) | $(ASAN)
	$(HOSTCXX) $(HOSTFLAGS) $(SAN) -c $< -o $@

$(ASAN)/librtpt.so: $(ASAN_HOST) $(BLD)/rt_kernel.o $(BLD)/rt_mis.o $(BLD)/rt_lbvh.o $(BLD)/rt_gsah.o
	$(HOSTCXX) -shared $(SAN) -o $@ $^ -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib

$(ASAN)/liboracle.so: oracle/pt_oracle.c oracle/pt_oracle.h include/rt_types.h | $(ASAN)
	$(HOSTCXX:clang++=clang) -x c -std=c11 -O1 -mfma -ffp-contract=off -fno-fast-math -fPIC -Wall -pthread \
	    $(SAN) -shared -o $@ oracle/pt_oracle.c -lm

asan: $(ASAN)/librtpt.so $(ASAN)/liboracle.so

asan-test: asan
	RTPT_SAN_DIR=$(abspath $(ASAN)) RTPT_SAN_RT=$(ASAN_RT) python3 tests/run_sanitized.py

clean:
	rm -rf $(BLD) $(ASAN) $(PKG)/librtpt.so $(PKG)/rtrace
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean asan asan-test
