# Build of the MI355X-native WeightedLD hot path.
#   make            -> weightedld_amd/libweightedld.so, weightedld_amd/bin/weighted_ld, oracle
# Everything is compiled for gfx950 only.  -ffp-contract=off: the LdStats
# epilogue must not be FMA-contracted (Rust never contracts); the pair kernels
# use explicit fmaf where a fused multiply-add is exact by construction.
# -fno-slp-vectorize: no packed-f32 VALU ops (v_pk_add/mul/fma_f32).  With them
# the one-plane pair kernel's f32 epilogue gave timing-dependent wrong values
# (one accumulator row, lanes 48-63) on MI355X; without them 16 repeated runs
# were bit-identical and oracle-exact ("packed-f32 epilogue");
# tests/test_codegen.py keeps them out of the built library.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := weightedld_amd
CSRC := $(PKG)/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Iinclude -I$(CSRC)
HIP_SRCS := $(CSRC)/encode.hip $(CSRC)/prepass.hip $(CSRC)/pair_valu.hip $(CSRC)/pair_mfma.hip \
            $(CSRC)/order.hip $(CSRC)/capi.hip
CXX_SRCS := $(CSRC)/host.cpp
HDRS := include/weightedld.h $(CSRC)/common.hpp $(CSRC)/kernels.hpp $(CSRC)/pair_common.hpp $(CSRC)/tile_order.hpp
OBJDIR := build/obj
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(CXX_SRCS))

all: $(PKG)/libweightedld.so $(PKG)/bin/weighted_ld oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) -x c++ -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC) -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(PKG)/libweightedld.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -lpthread

$(PKG)/bin/weighted_ld: $(CSRC)/cli.cpp $(CSRC)/tsv_format.hpp $(PKG)/libweightedld.so include/weightedld.h
	@mkdir -p $(PKG)/bin
	g++ -O2 -std=c++17 -Wall -Iinclude -I$(CSRC) -o $@ $(CSRC)/cli.cpp -L$(PKG) -lweightedld -Wl,-rpath,'$$ORIGIN/..' -lpthread

oracle:
	$(MAKE) -s -C oracle

# Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, this
# container): host.cpp (FASTA/VCF readers, filter, Henikoff) and cli.cpp built
# with g++ -fsanitize, linked with the unchanged gfx950 device objects; the host
# tests and the CLI's error paths then run against that build.
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
SANDIR := build/asan
DEV_OBJS := $(filter-out $(OBJDIR)/host.o,$(OBJS))

$(SANDIR)/host.o: $(CSRC)/host.cpp $(HDRS)
	@mkdir -p $(SANDIR)
	g++ $(SAN) -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC) -c $< -o $@

$(SANDIR)/libweightedld.so: $(DEV_OBJS) $(SANDIR)/host.o
	g++ -shared $(SAN) -o $@ $^ -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib

$(SANDIR)/weighted_ld: $(CSRC)/cli.cpp $(CSRC)/tsv_format.hpp $(SANDIR)/libweightedld.so include/weightedld.h
	g++ $(SAN) -std=c++17 -Wall -Iinclude -I$(CSRC) -o $@ $< -L$(SANDIR) -lweightedld -Wl,-rpath,'$$ORIGIN' -lpthread

sanitize: $(SANDIR)/libweightedld.so $(SANDIR)/weighted_ld oracle
	WLD_TEST_BUILD=$(SANDIR) ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
	LD_PRELOAD="$$(g++ -print-file-name=libasan.so) $$(g++ -print-file-name=libubsan.so)" \
	python3 -m pytest tests/test_host.py tests/test_tsv_format.py -q -m "not gpu" -p no:cacheprovider

clean:
	rm -rf build $(PKG)/libweightedld.so $(PKG)/bin
	$(MAKE) -s -C oracle clean

.PHONY: all clean oracle sanitize
