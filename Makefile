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

build/kernels/%.o: csrc/kernels/%.hip $(wildcard csrc/kernels/*.h)
	@mkdir -p build/kernels
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/kernels/%.o: csrc/kernels/%.cpp $(wildcard csrc/kernels/*.h)
	@mkdir -p build/kernels
	$(HIPCC) -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result -c $< -o $@

$(PKG)/_kernels.so: $(KOBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(KOBJ) -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib

build/runtime/%.o: csrc/runtime/%.cpp $(wildcard csrc/runtime/*.h)
	@mkdir -p build/runtime
	g++ $(CXXFLAGS) -c $< -o $@

$(PKG)/_runtime.so: $(ROBJ)
	g++ $(CXXFLAGS) -shared -o $@ $(ROBJ) -lpthread -lz -ldl

clean:
	rm -rf build $(PKG)/_kernels.so $(PKG)/_runtime.so

.PHONY: all clean
