# Builds the MI355X codec library in-tree (it travels to the GPU box with the
# snapshot) and the parity checker under oracle/.
#
#   make            -> coldforce_amd/libcfws.so + oracle/liboracle.so
#   make ref        -> also oracle/_ref/ (reference codec, needs /root/reference)

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
DEVSRC   := cfws_device cfws_h2 cfws_ops cfws_uniform
HOSTSRC  := cfws_frame cfws_pipeline cfws_index cfws_graph
HDR      := include/cfws.h include/cfws_co_ws_frame.h coldforce_amd/csrc/cfws_internal.h coldforce_amd/csrc/cfws_devpolicy.h
LIB      := coldforce_amd/libcfws.so
OBJDIR   := build

all: $(LIB) oracle examples guard

# test infrastructure: device buffers between unmapped guard ranges
# (tests/test_gpu_guard.py); host code only, no kernels
guard: tests/native/libguardmem.so

tests/native/libguardmem.so: tests/native/guardmem.cpp
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# C users of the ABI (no Python): built against include/, linked to libcfws.so
examples: build/examples/batch_roundtrip

build/examples/batch_roundtrip: examples/batch_roundtrip.c $(LIB) $(HDR)
	@mkdir -p build/examples
	$(CC) -O2 -std=gnu11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ $< \
	    -Lcoldforce_amd -lcfws -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../coldforce_amd' -Wl,-rpath,/opt/rocm/lib

$(OBJDIR)/%.o: coldforce_amd/csrc/%.hip $(HDR) coldforce_amd/csrc/cfws_kernels.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c $< -o $@

$(OBJDIR)/%.o: coldforce_amd/csrc/%.cpp $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c $< -o $@

$(LIB): $(addprefix $(OBJDIR)/,$(addsuffix .o,$(DEVSRC) $(HOSTSRC)))
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

oracle:
	$(MAKE) -s -C oracle

ref: all
	$(MAKE) -s -C oracle ref

asm: $(HDR) coldforce_amd/csrc/cfws_kernels.h
	@mkdir -p $(OBJDIR)/asm
	rm -f $(OBJDIR)/asm/resource-usage.txt
	for d in $(DEVSRC); do $(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c coldforce_amd/csrc/$$d.hip -o $(OBJDIR)/asm/$$d.o \
	    -save-temps=obj -Rpass-analysis=kernel-resource-usage 2>> $(OBJDIR)/asm/resource-usage.txt || exit 1; done

clean:
	rm -rf $(OBJDIR) $(LIB) tests/native/libguardmem.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle ref asm clean examples guard

# A/B build variants of the numeric tunables (kept out of git under build/): make variant V=ser4 F="-DCFWS_SER_LDS=40000"
variant: $(HDR)
	@mkdir -p $(OBJDIR)/variants/$(V)
	for d in $(DEVSRC); do $(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) $(F) -Iinclude -Icoldforce_amd/csrc -c coldforce_amd/csrc/$$d.hip -o $(OBJDIR)/variants/$(V)/$$d.o || exit 1; done
	for h in $(HOSTSRC); do $(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) $(F) -Iinclude -Icoldforce_amd/csrc -c coldforce_amd/csrc/$$h.cpp -o $(OBJDIR)/variants/$(V)/$$h.o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OBJDIR)/variants/libcfws_$(V).so $(OBJDIR)/variants/$(V)/*.o

.PHONY: variant
