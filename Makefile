# Top-level build: the HIP engine (gfx950), the DAG generator, the CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function
CC ?= gcc

ENGINE_SRC := $(wildcard babble_amd/csrc/engine/*.hip) $(wildcard babble_amd/csrc/engine/*.cpp)
ENGINE_HDR := $(wildcard babble_amd/csrc/engine/*.h) include/babble_hip.h

all: babble_amd/libbabble_gen.so babble_amd/libbabble_hip.so oracle/liboracle.so tests/cpp/hg_replay

babble_amd/libbabble_gen.so: babble_amd/csrc/dag_gen.c babble_amd/csrc/dag_gen.h
	$(CC) -O2 -fPIC -shared -Wall -Wno-deprecated-declarations -o $@ $< -lcrypto -lpthread

# one object per source (build/engine/*.o), so an edit rebuilds one file
ENGINE_OBJ := $(patsubst babble_amd/csrc/engine/%,build/engine/%.o,$(ENGINE_SRC))

build/engine/%.o: babble_amd/csrc/engine/% $(ENGINE_HDR)
	@mkdir -p build/engine
	$(HIPCC) $(HIPFLAGS) -Iinclude -c -o $@ $<

babble_amd/libbabble_hip.so: $(ENGINE_OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(ENGINE_OBJ) -L/opt/rocm/lib -lrccl -lcrypto -Wl,-rpath,/opt/rocm/lib

oracle/liboracle.so: oracle/hg_oracle.c oracle/hg_oracle.h
	$(MAKE) -C oracle

# C++ host mirror driver (plain g++; links the engine, rpath to the in-tree .so)
tests/cpp/hg_replay: tests/cpp/hg_replay.cpp include/babble_hashgraph.hpp include/babble_hip.h babble_amd/libbabble_hip.so
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -Lbabble_amd -lbabble_hip -Wl,-rpath,'$$ORIGIN/../../babble_amd'

# host-only AddressSanitizer build of the engine (tools/sanitize_engine.sh):
# the host files (api.cpp, frames.cpp) built by g++ with -fsanitize=address
# and UBSan, linked with the regular gfx950 kernel objects, loaded through
# BH_LIB_PATH with GCC's ASan runtime preloaded.  (clang's ROCm ASan runtime
# intercepts hsa_amd_memory_pool_allocate for device-side ASan, which needs
# XNACK, and fails the first device allocation here.)
HOST_SRC := $(wildcard babble_amd/csrc/engine/*.cpp)
KERNEL_OBJ := $(patsubst babble_amd/csrc/engine/%,build/engine/%.o,$(wildcard babble_amd/csrc/engine/*.hip))
ASAN_OBJ := $(patsubst babble_amd/csrc/engine/%,build/asan/%.o,$(HOST_SRC))
ASANFLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
build/asan/%.o: babble_amd/csrc/engine/% $(ENGINE_HDR)
	@mkdir -p build/asan
	$(CXX) $(ASANFLAGS) -std=c++17 -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -c -o $@ $<
tools/asan/libbabble_hip.so: $(ASAN_OBJ) $(KERNEL_OBJ)
	@mkdir -p tools/asan
	$(CXX) $(ASANFLAGS) -shared -o $@ $(ASAN_OBJ) $(KERNEL_OBJ) -L/opt/rocm/lib -lamdhip64 -lrccl -lcrypto -lpthread -Wl,-rpath,/opt/rocm/lib
asan: tools/asan/libbabble_hip.so

clean:
	rm -rf babble_amd/*.so oracle/*.so tests/cpp/hg_replay build/engine build/asan tools/asan

.PHONY: all asan clean
