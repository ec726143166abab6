# Build of the MI355X (gfx950) hot-path library.  `python -c "import __graft_entry__ as g; g.build()"`
# drives the same recipe.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
HIPFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-result

LIB  = v2e2v_amd/libcista_hip.so
SRCS = v2e2v_amd/csrc/cista_abi.hip
DEPS = $(SRCS) v2e2v_amd/csrc/cista_kernels.hpp v2e2v_amd/csrc/cista_backward.hpp include/cista_lstc.h

all: $(LIB)

$(LIB): $(DEPS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

clean:
	rm -f $(LIB)

.PHONY: all clean
