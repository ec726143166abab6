# Build of the MI355X (gfx950) hot-path library.  `python -c "import __graft_entry__ as g; g.build()"`
# runs this Makefile.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
HIPFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-result

LIB  = v2e2v_amd/libcista_hip.so
OBJ  = build/cista_abi.o build/cista_voxel.o build/cista_ssim.o build/cista_v2e.o

all: $(LIB)

build/cista_abi.o: v2e2v_amd/csrc/cista_abi.hip v2e2v_amd/csrc/cista_kernels.hpp \
                   v2e2v_amd/csrc/cista_backward.hpp include/cista_lstc.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/cista_voxel.o: v2e2v_amd/csrc/cista_voxel.hip include/cista_voxel.h include/cista_lstc.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/cista_ssim.o: v2e2v_amd/csrc/cista_ssim.hip include/cista_loss.h include/cista_lstc.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/cista_v2e.o: v2e2v_amd/csrc/cista_v2e.hip include/cista_v2e.h include/cista_voxel.h include/cista_lstc.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
