# libgfslam (HIP, gfx950) + the CPU oracle (test infrastructure).
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
ARCH    ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
           -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function
ORCFLAGS = -O3 -fno-tree-vectorize -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function

CSRC    = gf_orb_slam_amd/csrc
HIPSRCS = $(wildcard $(CSRC)/*.hip)
HIPOBJS = $(patsubst $(CSRC)/%.hip,build/%.o,$(HIPSRCS))
CPPSRCS = $(wildcard $(CSRC)/*.cpp)
CPPOBJS = $(patsubst $(CSRC)/%.cpp,build/%.cpp.o,$(CPPSRCS))
HDRS    = $(wildcard $(CSRC)/*.h) include/gfslam/abi.h include/gfslam/orbslam.h
LIB     = gf_orb_slam_amd/libgfslam.so

ORCSRCS = $(wildcard oracle/*.cpp)
ORCLIB  = oracle/liboracle.so

all: $(LIB) $(ORCLIB)

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build
	$(CXX) -O3 -fno-tree-vectorize -std=c++17 -fPIC -ffp-contract=off -Wall -c $< -o $@

$(LIB): $(HIPOBJS) $(CPPOBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -L/opt/rocm/lib -lrccl -o $@

$(ORCLIB): $(ORCSRCS) $(wildcard oracle/*.h) $(CSRC)/orb_pattern.h $(CSRC)/select.h $(CSRC)/libm_sincosf.h include/gfslam/abi.h
	$(CXX) $(ORCFLAGS) -shared $(ORCSRCS) -o $@ -lpthread

# timing copy of the oracle for bench.py's cpu_baseline: vectorisation on,
# AVX2-class target (portable to the GPU node's host), same arithmetic order
ORCFAST = oracle/liboracle_fast.so
all: $(ORCFAST)
$(ORCFAST): $(ORCSRCS) $(wildcard oracle/*.h) $(CSRC)/orb_pattern.h $(CSRC)/select.h $(CSRC)/libm_sincosf.h include/gfslam/abi.h
	$(CXX) -O3 -march=x86-64-v3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -shared $(ORCSRCS) -o $@ -lpthread

clean:
	rm -rf build $(LIB) $(ORCLIB) $(ORCFAST)

.PHONY: all clean

SELCHECK = tests/helpers/libselcheck.so
all: $(SELCHECK)
$(SELCHECK): tests/helpers/select_check.cpp $(CSRC)/select.h
	$(CXX) -O2 -std=c++17 -fPIC -shared $< -o $@

# C++ drop-in layer driver (tests/test_dropin_gpu.py runs it on the GPU box)
DROPIN = tests/cpp/dropin_frontend
all: $(DROPIN)
$(DROPIN): tests/cpp/dropin_frontend.cpp include/gfslam/orbslam.h include/gfslam/abi.h $(LIB)
	$(CXX) -O2 -std=c++17 -Iinclude $< -Lgf_orb_slam_amd -lgfslam -Wl,-rpath,'$$ORIGIN/../../gf_orb_slam_amd' -o $@

# C-ABI-only caller: batched front-end sequence + local BA (tests/test_dropin_gpu.py)
SEQDRV = tests/cpp/sequence_driver
all: $(SEQDRV)
$(SEQDRV): tests/cpp/sequence_driver.cpp include/gfslam/orbslam.h include/gfslam/abi.h $(LIB)
	$(CXX) -O2 -std=c++17 -Iinclude $< -Lgf_orb_slam_amd -lgfslam -Wl,-rpath,'$$ORIGIN/../../gf_orb_slam_amd' -o $@

# diagnostic build: k_active_match phase stamps (scripts/am_stamps.py), never the product
STAMPLIB = gf_orb_slam_amd/diag/libgfslam_am.so
stamp: $(STAMPLIB)
build/stamp/gf.o: $(CSRC)/gf.hip $(HDRS)
	@mkdir -p build/stamp
	$(HIPCC) $(HIPFLAGS) -DGF_AM_STAMP -c $< -o $@
$(STAMPLIB): build/stamp/gf.o $(filter-out build/gf.o,$(HIPOBJS)) $(CPPOBJS) | gf_orb_slam_amd/diag
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -L/opt/rocm/lib -lrccl -o $@
gf_orb_slam_amd/diag:
	mkdir -p $@
.PHONY: stamp
