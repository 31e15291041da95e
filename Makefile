# Build everything in-tree (the built .so / binaries travel to the GPU box with gpurun).
#   make            libsheep_hip.so + CLIs + oracle (+ oracle/_ref if /root/reference exists)
#   make hip        sheep_amd/lib/libsheep_hip.so (gfx950 only)
#   make cli        sheep_amd/bin/{graph2tree,partition_tree,merge_trees,degree_sequence,rmat_gen}
#   make oracle     oracle/lib/libsheep_oracle.so (test infrastructure)
#   make ref        oracle/_ref/* (reference sources compiled in place; container only)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
JOBS    ?= 8
HIPFLAGS:= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-value \
           -Iinclude -Isheep_amd/csrc
HIPSRC  := $(wildcard sheep_amd/csrc/*.hip)
HIPOBJ  := $(patsubst sheep_amd/csrc/%.hip,build/hip/%.o,$(HIPSRC))
HIPHDR  := $(wildcard sheep_amd/csrc/*.hpp) include/sheep_hip.h
LIB     := sheep_amd/lib/libsheep_hip.so
CLIS    := graph2tree partition_tree merge_trees degree_sequence
CLIBIN  := $(addprefix sheep_amd/bin/,$(CLIS))
CXX     ?= g++

all: hip cli oracle ref

hip: $(LIB)

build/hip/%.o: sheep_amd/csrc/%.hip $(HIPHDR)
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIPOBJ)
	@mkdir -p sheep_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIPOBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

cli: $(CLIBIN)

sheep_amd/bin/%: sheep_amd/cli/%.cpp $(LIB) $(wildcard sheep_amd/include/sheep/*.hpp) include/sheep_hip.h
	@mkdir -p sheep_amd/bin
	$(CXX) -std=c++17 -O2 -Wall -Iinclude -Isheep_amd/include -o $@ $< \
	    -Lsheep_amd/lib -lsheep_hip -Wl,-rpath,'$$ORIGIN/../lib'

oracle: oracle/lib/libsheep_oracle.so

oracle/lib/libsheep_oracle.so: oracle/sheep_oracle.cpp
	@mkdir -p oracle/lib
	$(CXX) -std=c++17 -O2 -fopenmp -fPIC -shared -Wall -o $@ $<

ref:
	@if [ -d /root/reference/lib ]; then $(MAKE) -C oracle/ref; else echo "no /root/reference: skipping oracle/_ref"; fi

clean:
	rm -rf build sheep_amd/lib sheep_amd/bin oracle/lib

.PHONY: all hip cli oracle ref clean

# A kernel variant for A/B runs: make variant V=name DEFS="-DFOO=1" -> sheep_amd/lib/variants/libsheep_hip_$(V).so
# (bench.py / tests load it with SHEEP_HIP_LIB=...)
variant:
	@mkdir -p build/var_$(V) sheep_amd/lib/variants
	for f in $(HIPSRC); do $(HIPCC) $(HIPFLAGS) $(DEFS) -c $$f -o build/var_$(V)/$$(basename $$f .hip).o & done; wait
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o sheep_amd/lib/variants/libsheep_hip_$(V).so build/var_$(V)/*.o \
	    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: variant
