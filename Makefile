# libhpnn (MI355X-native) build.
#   make            -> hpnn_amd/lib/libhpnn.so, bin/train_nn, bin/run_nn,
#                      bin/pmnist, bin/pdif, hpnn_amd/_native*.so
#   make clean
#   make install PREFIX=/usr/local  -> lib/libhpnn.so, include/libhpnn.h + include/libhpnn/*.h,
#                                      lib/pkgconfig/libhpnn.pc, bin/{train_nn,run_nn,...}
# Device code: hipcc --offload-arch=gfx950 only (no other targets).
ROCM      ?= /opt/rocm
ARCH      ?= gfx950
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
PYTHON    ?= python3
BUILD     := build
LIBDIR    := hpnn_amd/lib
BINDIR    := bin

INC       := -Iinclude -I$(ROCM)/include
DEFS      := -D__HIP_PLATFORM_AMD__
# -ffp-contract=off keeps the FP64 CPU oracle bit-stable across compilers
CXXFLAGS  := -O2 -std=c++17 -fPIC -fopenmp -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result $(INC) $(DEFS)
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics $(INC)
# make ABLATIONS=1: also build the front kernels' profiling ablations (HPNN_TILE_ABL /
# HPNN_WIDE_ABL, wrong results by design); the default library has none of them
HIPFLAGS  += $(if $(ABLATIONS),-DHPNN_ABLATIONS)
LDFLAGS   := -L$(ROCM)/lib -lamdhip64 -fopenmp

CORE_SRC  := $(wildcard csrc/core/*.cpp) $(wildcard csrc/cpu/*.cpp) $(wildcard csrc/dist/*.cpp) csrc/gpu/gpu_engine.cpp csrc/gpu/tp_engine.cpp csrc/gpu/bplan.cpp
HIP_SRC   := $(wildcard csrc/gpu/*.hip) $(wildcard csrc/dist/*.hip)
CORE_OBJ  := $(patsubst %.cpp,$(BUILD)/%.o,$(CORE_SRC))
HIP_OBJ   := $(patsubst %.hip,$(BUILD)/%.o,$(HIP_SRC))
HDRS      := $(wildcard include/*.h include/libhpnn/*.h csrc/*/*.h)

PYEXT     := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC     := $(shell $(PYTHON) -c "import sysconfig,pybind11;print('-I'+sysconfig.get_paths()['include'],'-I'+pybind11.get_include())")
PYMOD     := hpnn_amd/_native$(PYEXT)

LIB       := $(LIBDIR)/libhpnn.so
BINS      := $(BINDIR)/train_nn $(BINDIR)/run_nn $(BINDIR)/pmnist $(BINDIR)/pdif $(BINDIR)/pack_nn

all: $(LIB) $(BINS) $(PYMOD)

$(BUILD)/%.o: %.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# device objects depend on the device flags: a change (e.g. make ABLATIONS=1, then plain make)
# rewrites this stamp at parse time and rebuilds them, so an ablation build never stays behind
HIPSTAMP  := $(BUILD)/.hipflags
_stamp    := $(shell mkdir -p $(BUILD); echo '$(HIPFLAGS)' | cmp -s - $(HIPSTAMP) || echo '$(HIPFLAGS)' > $(HIPSTAMP))

$(BUILD)/%.o: %.hip $(HDRS) $(HIPSTAMP)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CORE_OBJ) $(HIP_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ $(LDFLAGS) -Wl,-soname,libhpnn.so

$(BINDIR)/%: tools/%.cpp $(LIB) tools/cli_common.h Makefile
	@mkdir -p $(BINDIR)
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -lhpnn $(LDFLAGS) -Wl,-rpath,'$$ORIGIN/../$(LIBDIR):$$ORIGIN/../lib'

$(PYMOD): csrc/python/bind.cpp $(LIB) $(HDRS)
	$(CXX) $(CXXFLAGS) -shared $(PYINC) $< -o $@ -L$(LIBDIR) -lhpnn $(LDFLAGS) -Wl,-rpath,'$$ORIGIN/lib'

clean:
	rm -rf $(BUILD) $(LIB) $(BINS) $(PYMOD)

# Installation (the reference's src/Makefile.am:12-41 layout: libhpnn.h in include/, the
# other headers in include/libhpnn/, pkg-config file in lib/pkgconfig/).  The CLIs find
# the installed library through their $$ORIGIN/../lib rpath.
PREFIX    ?= /usr/local
VERSION   := 0.3.0
install: $(LIB) $(BINS)
	install -d $(DESTDIR)$(PREFIX)/lib/pkgconfig $(DESTDIR)$(PREFIX)/include/libhpnn $(DESTDIR)$(PREFIX)/bin
	install -m 755 $(LIB) $(DESTDIR)$(PREFIX)/lib/libhpnn.so
	install -m 644 include/libhpnn.h $(DESTDIR)$(PREFIX)/include/libhpnn.h
	install -m 644 include/libhpnn/*.h $(DESTDIR)$(PREFIX)/include/libhpnn/
	install -m 755 $(BINS) $(DESTDIR)$(PREFIX)/bin/
	sed -e 's|@PREFIX@|$(PREFIX)|' -e 's|@ROCM@|$(ROCM)|' -e 's|@VERSION@|$(VERSION)|' libhpnn.pc.in \
	    > $(DESTDIR)$(PREFIX)/lib/pkgconfig/libhpnn.pc

uninstall:
	rm -f $(DESTDIR)$(PREFIX)/lib/libhpnn.so $(DESTDIR)$(PREFIX)/include/libhpnn.h \
	      $(DESTDIR)$(PREFIX)/lib/pkgconfig/libhpnn.pc $(addprefix $(DESTDIR)$(PREFIX)/bin/,$(notdir $(BINS)))
	rm -rf $(DESTDIR)$(PREFIX)/include/libhpnn

.PHONY: all clean install uninstall

# Host-side sanitizer build (AddressSanitizer + UBSan) of the C API, CPU engine, runtime,
# comm layer and CLIs; device code objects are the regular ones (GPU sanitizers are not
# available on this pool).  tests/test_sanitizers_cpu.py runs the CPU workflows under it.
ASAN_DIR   := $(BUILD)/asan
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
ASAN_OBJ   := $(patsubst %.cpp,$(ASAN_DIR)/%.o,$(CORE_SRC))
ASAN_BINS  := $(ASAN_DIR)/train_nn $(ASAN_DIR)/run_nn $(ASAN_DIR)/pack_nn

$(ASAN_DIR)/%.o: %.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) -c $< -o $@

$(ASAN_DIR)/%: tools/%.cpp $(ASAN_OBJ) $(HIP_OBJ) tools/cli_common.h
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) $< $(ASAN_OBJ) $(HIP_OBJ) -o $@ $(LDFLAGS) -ldl

asan: $(ASAN_BINS)

.PHONY: asan
