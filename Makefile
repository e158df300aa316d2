# Builds the gfx950 kernel library (ctypes C ABI) and the native runtime (TFRecord IO, prefetcher).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics -Wno-unused-result
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
PKG := homebrewnlp_mtf_amd
KSRC := $(wildcard csrc/kernels/*.hip)
KCPP := $(wildcard csrc/kernels/*.cpp)
KOBJ := $(patsubst csrc/kernels/%.hip,build/kernels/%.o,$(KSRC)) $(patsubst csrc/kernels/%.cpp,build/kernels/%.o,$(KCPP))
RSRC := $(wildcard csrc/runtime/*.cpp)
ROBJ := $(patsubst csrc/runtime/%.cpp,build/runtime/%.o,$(RSRC))

all: $(PKG)/_kernels.so $(if $(RSRC),$(PKG)/_runtime.so,)

# attention: no SLP vectorisation -- adjacent f32 adds / multiplies packed into v_pk_*_f32 cost more issue cycles
# than two scalar ops beside MFMAs (MI355X_MICROARCH.md, 'price of one filler beside MFMAs')
build/kernels/attention.o: HIPFLAGS += -fno-slp-vectorize
# attention-map kernels: MFMAs in the VGPR form -- the AGPR form kept the output accumulators in VGPRs across the
# key loop and moved all of them into AGPRs and back every tile (profiles/r5_attn_map.md)
build/kernels/attn_map.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form

build/kernels/%.o: csrc/kernels/%.hip $(wildcard csrc/kernels/*.h)
	@mkdir -p build/kernels
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/kernels/%.o: csrc/kernels/%.cpp $(wildcard csrc/kernels/*.h)
	@mkdir -p build/kernels
	$(HIPCC) -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result -c $< -o $@

$(PKG)/_kernels.so: $(KOBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(KOBJ)

build/runtime/%.o: csrc/runtime/%.cpp $(wildcard csrc/runtime/*.h)
	@mkdir -p build/runtime
	g++ $(CXXFLAGS) -c $< -o $@

$(PKG)/_runtime.so: $(ROBJ)
	g++ $(CXXFLAGS) -shared -o $@ $(ROBJ) -lpthread -lz -ldl

# Sanitizer builds of the threaded host runtime, loaded through OBST_RUNTIME_SO into a stock python
# with the sanitizer runtime preloaded; `make sancheck` runs the data / runtime CPU tests under both.
SAN_CXX := g++ -O1 -g -std=c++17 -fPIC -fno-omit-frame-pointer -Wall -Wno-unused-result
build/san/_runtime_asan.so: $(RSRC) $(wildcard csrc/runtime/*.h)
	@mkdir -p build/san
	$(SAN_CXX) -fsanitize=address,undefined -shared -o $@ $(RSRC) -lpthread -lz -ldl
build/san/_runtime_tsan.so: $(RSRC) $(wildcard csrc/runtime/*.h)
	@mkdir -p build/san
	$(SAN_CXX) -fsanitize=thread -shared -o $@ $(RSRC) -lpthread -lz -ldl
asan: build/san/_runtime_asan.so
tsan: build/san/_runtime_tsan.so
SAN_TESTS ?= tests/test_data.py tests/test_runtime_cpu.py
# under TSan only the tests that drive the native runtime in-process (the REST / subprocess tests spawn uninstrumented
# interpreters and threads that TSan slows to a crawl)
TSAN_K ?= not rest_api and not debug_mode and not kv_cache and not fault_injection
sancheck: asan tsan
	OBST_RUNTIME_SO=$(CURDIR)/build/san/_runtime_asan.so LD_PRELOAD="$$(g++ -print-file-name=libasan.so) $$(g++ -print-file-name=libubsan.so)" \
	  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	  python -m pytest -q -x -m "not gpu" -p no:cacheprovider $(SAN_TESTS)
	OBST_RUNTIME_SO=$(CURDIR)/build/san/_runtime_tsan.so LD_PRELOAD="$$(g++ -print-file-name=libtsan.so)" \
	  TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
	  python -m pytest -q -x -m "not gpu" -p no:cacheprovider $(SAN_TESTS) -k "$(TSAN_K)"

clean:
	rm -rf build $(PKG)/_kernels.so $(PKG)/_runtime.so

.PHONY: all clean asan tsan sancheck
