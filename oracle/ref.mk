# ref.mk -- TEST INFRASTRUCTURE ONLY: builds oracle/_ref/libpgn_ref.so, the reference's own svb16
# split/merge code for every compile-time variant, compiled from the sources where they lie under
# /root/reference (nothing is copied into this repository; outputs go to oracle/_ref/ only, which is
# git-ignored).
#
# For each variant header (pod5/c++/pod5_format/pgnano/svb16/{C5,C4,C3,C2,C1,VBZ_0}.hpp) the block
# from its extern statistics declarations through `} // namespace svb16` is extracted VERBATIM with sed
#   C5.hpp:27-277  C4.hpp:27-269  C3.hpp:27-208  C2.hpp:27-191  C1.hpp:31-197  VBZ_0.hpp:30-311
# and piped on stdin to g++ between ref/ref_prelude.hpp (the reference's own common.hpp, svb16.h,
# encode_scalar.hpp, decode_scalar.hpp and the vendored gsl-lite) and ref/ref_api.inc (our extern "C"
# wrappers).  The rest of those headers (the pgnano:: compress/decompress bodies) needs arrow, the
# CMake-generated pod5_format_export.h and BAM_handler.h (boost + htslib): not built.
#
#   make -f ref.mk            (from oracle/; a no-op when /root/reference is absent)
REF ?= /root/reference
SVB := $(REF)/pod5/c++/pod5_format/pgnano/svb16
GSL := $(REF)/pod5/third_party/include
OUT := _ref
CXX ?= g++
CXXFLAGS ?= -O2 -fPIC -std=c++17 -w
INC := -I ref -I $(SVB) -I $(GSL)
FRAG = sed -n '/^extern long full_size_keys/,/^} \/\/ namespace svb16/p' $(SVB)/$(1).hpp

VARIANTS := C5 C4 C3 C2 C1 VBZ0
OBJS := $(addprefix $(OUT)/,$(addsuffix .o,$(VARIANTS)) counters.o)

ifeq ($(wildcard $(SVB)/C5.hpp),)
all:
	@echo "ref.mk: $(SVB) not present; oracle/_ref not built"
else
all: $(OUT)/libpgn_ref.so $(OUT)/libpgn_ref_vbz.so
endif

$(OUT)/libpgn_ref.so: $(OBJS)
	$(CXX) -shared -o $@ $^

# the pod5 VBZ codec's svb16 stage, included directly from pod5/c++/pod5_format/svb16/ (SSE4.1 decode
# path as the reference builds it on x86-64)
$(OUT)/libpgn_ref_vbz.so: ref/ref_vbz.cpp
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -msse4.1 -mssse3 -I $(REF)/pod5/c++/pod5_format -I $(GSL) -shared -o $@ $<

$(OUT)/counters.o: ref/ref_counters.cpp
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

# header name of a variant (VBZ0 lives in VBZ_0.hpp)
hdr = $(if $(filter VBZ0,$(1)),VBZ_0,$(1))

$(OUT)/%.o: ref/ref_prelude.hpp ref/ref_api.inc
	@mkdir -p $(OUT)
	{ echo '#include "ref_prelude.hpp"'; $(call FRAG,$(call hdr,$*)); echo '#include "ref_api.inc"'; } \
	  | $(CXX) $(CXXFLAGS) -DREF_$* $(INC) -x c++ -c -o $@ -

clean:
	rm -rf $(OUT)

.PHONY: all clean
