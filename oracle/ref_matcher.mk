# Compiles the REFERENCE's own 32-test matcher from its source file where it lies -- the two
# functions of /root/reference/feature_matching_parallel/feature_matching_parallel.cpp:39-113
# (hammingDistance + matchCustomBinaryDescriptorsThreadPool), cut out at build time into the
# git- and gpurun-ignored build/ directory, never copied into this repo -- together with the
# reference's own std-only thread pool (feature_extraction_parallel/threadpool.h, ts_queue.h,
# join_threads.h, included from /root/reference).  The rest of that .cpp needs OpenCV (its includes
# :14-17 and the debug helpers :115-163), so only the two functions are taken; no stand-in header
# is written.  Output: oracle/_ref/libref_matcher.so (git-ignored), loaded by tests/test_ref_matcher.py
# as the checker of the oracle's voo_match (and through it k_match).
REF    ?= /root/reference
SRC    := $(REF)/feature_matching_parallel/feature_matching_parallel.cpp
POOL   := $(REF)/feature_extraction_parallel
HERE   := $(dir $(lastword $(MAKEFILE_LIST)))
OUT    := $(HERE)_ref
TMP    := $(HERE)../build/ref_matcher
CXX    ?= g++

all: $(OUT)/libref_matcher.so

# the two functions: from `inline int hammingDistance` to the line before `findCommonMatches`
$(TMP)/matcher_body.inc: $(SRC)
	@mkdir -p $(TMP)
	awk '/^inline int hammingDistance/{p=1} /^std::vector<std::pair<int, int>> findCommonMatches/{p=0} p' $< > $@
	@grep -q '^std::vector<std::pair<int, int>> matchCustomBinaryDescriptorsThreadPool(' $@ || { echo "matcher not found in $<"; rm -f $@; exit 1; }

$(OUT)/libref_matcher.so: $(HERE)ref_matcher_drv.cpp $(TMP)/matcher_body.inc $(POOL)/threadpool.h $(POOL)/ts_queue.h $(POOL)/join_threads.h
	@mkdir -p $(OUT)
	$(CXX) -O2 -std=c++17 -fPIC -shared -pthread -I$(POOL) -I$(TMP) -o $@ $(HERE)ref_matcher_drv.cpp

clean:
	rm -f $(OUT)/libref_matcher.so $(TMP)/matcher_body.inc

.PHONY: all clean
