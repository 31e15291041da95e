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

# CPU sanitizer builds (host code only — no GPU sanitizer on this pool):
#   make asan        oracle/lib/asan/libsheep_oracle.so, sheep_amd/lib/asan/libsheep_hip.so (host code
#                    under -fsanitize=address,undefined, device code as usual) and the CLIs against it
#   make asan-check  the CPU suite (pytest -m "not gpu") with those builds loaded, ASan's runtime
#                    preloaded into the test process; log in profiles/r5/asan_cpu_suite.log
# One compiler for everything (clang: ROCm's llvm), so one sanitizer runtime serves all.
CLANG   := /opt/rocm/lib/llvm/bin/clang++
ASANRT  := $(firstword $(wildcard /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so))
SANFLAGS:= -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -shared-libasan
HIPSAN  := $(foreach f,$(SANFLAGS),-Xarch_host $(f))
ASANOBJ := $(patsubst sheep_amd/csrc/%.hip,build/asan/%.o,$(HIPSRC))

asan: oracle/lib/asan/libsheep_oracle.so sheep_amd/lib/asan/libsheep_hip.so $(addprefix sheep_amd/bin/asan/,$(CLIS))

oracle/lib/asan/libsheep_oracle.so: oracle/sheep_oracle.cpp
	@mkdir -p oracle/lib/asan
	$(CLANG) -std=c++17 -O1 -fopenmp -fPIC -shared $(SANFLAGS) -o $@ $< -L/opt/rocm/lib/llvm/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib

build/asan/%.o: sheep_amd/csrc/%.hip $(HIPHDR)
	@mkdir -p build/asan
	$(HIPCC) $(HIPFLAGS) $(HIPSAN) -c $< -o $@

sheep_amd/lib/asan/libsheep_hip.so: $(ASANOBJ)
	@mkdir -p sheep_amd/lib/asan
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(HIPSAN) -o $@ $(ASANOBJ) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

sheep_amd/bin/asan/%: sheep_amd/cli/%.cpp sheep_amd/lib/asan/libsheep_hip.so $(wildcard sheep_amd/include/sheep/*.hpp) include/sheep_hip.h
	@mkdir -p sheep_amd/bin/asan
	$(CLANG) -std=c++17 -O1 $(SANFLAGS) -Iinclude -Isheep_amd/include -o $@ $< \
	    -Lsheep_amd/lib/asan -lsheep_hip -Wl,-rpath,'$$ORIGIN/../../lib/asan'

asan-check: asan
	@mkdir -p profiles/r5
	@for f in oracle/lib/asan/libsheep_oracle.so sheep_amd/lib/asan/libsheep_hip.so sheep_amd/bin/asan/graph2tree; do \
	  echo "$$f: $$(nm -D --undefined-only $$f | grep -c __asan_report) ASan report hooks, $$(nm -D --undefined-only $$f | grep -c __ubsan_handle) UBSan handlers"; \
	done > profiles/r5/asan_cpu_suite.log
	bash -o pipefail -c 'LD_PRELOAD=$(ASANRT) ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
	  SHEEP_ORACLE_LIB=$(CURDIR)/oracle/lib/asan/libsheep_oracle.so SHEEP_HIP_LIB=$(CURDIR)/sheep_amd/lib/asan/libsheep_hip.so \
	  SHEEP_BIN_DIR=$(CURDIR)/sheep_amd/bin/asan \
	  python -m pytest tests -v -m "not gpu" -p no:cacheprovider 2>&1 | tee -a profiles/r5/asan_cpu_suite.log'

.PHONY: asan asan-check

.PHONY: all hip cli oracle ref clean

# A kernel variant for A/B runs: make variant V=name DEFS="-DFOO=1" -> sheep_amd/lib/variants/libsheep_hip_$(V).so
# (bench.py / tests load it with SHEEP_HIP_LIB=...)
variant:
	@mkdir -p build/var_$(V) sheep_amd/lib/variants
	for f in $(HIPSRC); do $(HIPCC) $(HIPFLAGS) $(DEFS) -c $$f -o build/var_$(V)/$$(basename $$f .hip).o & done; wait
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o sheep_amd/lib/variants/libsheep_hip_$(V).so build/var_$(V)/*.o \
	    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
.PHONY: variant
