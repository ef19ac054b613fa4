# Build recipe (no cmake): hipcc for the product library, gcc for the oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
LIB = regex_amd/lib/librure_amd.so
HOST_SRC = regex_amd/csrc/host/syntax.cpp regex_amd/csrc/host/compile.cpp regex_amd/csrc/host/dfa_build.cpp \
           regex_amd/csrc/host/nfa_build.cpp regex_amd/csrc/host/literals.cpp \
           regex_amd/csrc/host/literal_sets.cpp regex_amd/csrc/host/knobs.cpp
RT_SRC = regex_amd/csrc/build.cpp regex_amd/csrc/dispatch.cpp regex_amd/csrc/scratch.cpp regex_amd/csrc/capi.cpp
RT_OBJ = $(patsubst regex_amd/csrc/%.cpp,$(OBJDIR)/rt_%.o,$(RT_SRC))
KERNEL_SRC = regex_amd/csrc/kernels/dfa_scan.hip regex_amd/csrc/kernels/nfa_scan.hip regex_amd/csrc/kernels/iter_scan.hip \
             regex_amd/csrc/kernels/replace_scan.hip regex_amd/csrc/kernels/gather_scan.hip \
             regex_amd/csrc/kernels/match_types.hip regex_amd/csrc/kernels/big_dfa.hip \
             regex_amd/csrc/kernels/run_iter.hip
KERNEL_OBJ = $(patsubst regex_amd/csrc/kernels/%.hip,$(OBJDIR)/%.o,$(KERNEL_SRC))
HDRS = $(wildcard regex_amd/csrc/host/*.hpp regex_amd/csrc/host/*.h regex_amd/csrc/kernels/*.hpp include/*.h)
OBJDIR = regex_amd/build
HOST_OBJ = $(patsubst regex_amd/csrc/host/%.cpp,$(OBJDIR)/%.o,$(HOST_SRC))

ORACLE_LIB = oracle/build/liboracle.so
ORACLE_SRC = $(wildcard oracle/*.c)

all: $(LIB) $(ORACLE_LIB)

# host code: no device pass (hipcc would otherwise also compile it for a default GPU)
$(OBJDIR)/%.o: regex_amd/csrc/host/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) --offload-host-only -c $< -o $@

$(OBJDIR)/rt_%.o: regex_amd/csrc/%.cpp $(HDRS) regex_amd/csrc/runtime.hpp
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) --offload-host-only -c $< -o $@

$(OBJDIR)/%.o: regex_amd/csrc/kernels/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) --offload-arch=$(ARCH) -c $< -o $@

$(LIB): $(HOST_OBJ) $(RT_OBJ) $(KERNEL_OBJ)
	@mkdir -p regex_amd/lib
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

$(ORACLE_LIB): $(ORACLE_SRC) $(wildcard oracle/*.h)
	@mkdir -p oracle/build
	gcc -O3 -std=c11 -fPIC -shared -Wall -o $@ $(ORACLE_SRC) -lpthread

# diagnostic A/B library (tools/*): make ab AB=<name> ABFLAGS=-D...
ab:
	@mkdir -p regex_amd/build/ab_$(AB) regex_amd/lib
	$(MAKE) LIB=regex_amd/lib/librure_amd_$(AB).so OBJDIR=regex_amd/build/ab_$(AB) CXXFLAGS="$(CXXFLAGS) $(ABFLAGS)" regex_amd/lib/librure_amd_$(AB).so

clean:
	rm -rf regex_amd/build regex_amd/lib oracle/build

.PHONY: all clean ab
