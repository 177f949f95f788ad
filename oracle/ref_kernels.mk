# Compiles the REFERENCE's own OpenCL extract kernels from their source file where it lies
# (/root/reference/kernels/feature_extraction_kernel_functions.c, never copied into this
# repo) into gfx950 code objects under oracle/_ref/ (git-ignored; travels to the GPU box
# with the snapshot).  tests/test_ref_kernels.py loads them through the ROCm OpenCL
# runtime (clCreateProgramWithBinary) and checks the CPU oracle against them.
#
#   strict: no contraction, correctly rounded f32 divide/sqrt -- the arithmetic contract
#           this project fixes; expected bit-exact vs the oracle
#   stock : clang's OpenCL defaults (contraction on, relaxed divide/sqrt), the closest
#           offline stand-in for the reference's clBuildProgram with no options
#           (feature_extraction_parallel_GPU.cpp:105); differences are reported, not failed
REF    ?= /root/reference
SRC    := $(REF)/kernels/feature_extraction_kernel_functions.c
CLANG  ?= /opt/rocm/lib/llvm/bin/clang
OUT    := $(dir $(lastword $(MAKEFILE_LIST)))_ref
CLFLAGS := -x cl -cl-std=CL1.2 -target amdgcn-amd-amdhsa -mcpu=gfx950 -O3

all: $(OUT)/fe_kernels_strict.co $(OUT)/fe_kernels_stock.co

$(OUT)/fe_kernels_strict.co: $(SRC)
	@mkdir -p $(OUT)
	$(CLANG) $(CLFLAGS) -ffp-contract=off -cl-fp32-correctly-rounded-divide-sqrt $< -o $@

$(OUT)/fe_kernels_stock.co: $(SRC)
	@mkdir -p $(OUT)
	$(CLANG) $(CLFLAGS) $< -o $@

clean:
	rm -f $(OUT)/fe_kernels_strict.co $(OUT)/fe_kernels_stock.co

.PHONY: all clean
