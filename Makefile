# Builds the MI355X codec library in-tree (it travels to the GPU box with the
# snapshot) and the parity checker under oracle/.
#
#   make            -> coldforce_amd/libcfws.so + oracle/liboracle.so
#   make ref        -> also oracle/_ref/ (reference codec, needs /root/reference)

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
HOSTSRC  := cfws_frame cfws_pipeline cfws_index cfws_graph
HDR      := include/cfws.h include/cfws_co_ws_frame.h coldforce_amd/csrc/cfws_internal.h
LIB      := coldforce_amd/libcfws.so
OBJDIR   := build

all: $(LIB) oracle examples

# C users of the ABI (no Python): built against include/, linked to libcfws.so
examples: build/examples/batch_roundtrip

build/examples/batch_roundtrip: examples/batch_roundtrip.c $(LIB) $(HDR)
	@mkdir -p build/examples
	$(CC) -O2 -std=gnu11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -o $@ $< \
	    -Lcoldforce_amd -lcfws -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../coldforce_amd' -Wl,-rpath,/opt/rocm/lib

$(OBJDIR)/cfws_device.o: coldforce_amd/csrc/cfws_device.hip $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c $< -o $@

$(OBJDIR)/%.o: coldforce_amd/csrc/%.cpp $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c $< -o $@

$(LIB): $(OBJDIR)/cfws_device.o $(addprefix $(OBJDIR)/,$(addsuffix .o,$(HOSTSRC)))
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

oracle:
	$(MAKE) -s -C oracle

ref: all
	$(MAKE) -s -C oracle ref

asm: coldforce_amd/csrc/cfws_device.hip $(HDR)
	@mkdir -p $(OBJDIR)/asm
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -Iinclude -Icoldforce_amd/csrc -c $< -o $(OBJDIR)/asm/cfws_device.o \
	    -save-temps=obj -Rpass-analysis=kernel-resource-usage 2> $(OBJDIR)/asm/resource-usage.txt

clean:
	rm -rf $(OBJDIR) $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle ref asm clean examples

# A/B build variants (kept out of git under build/): make variant V=nt F="-DCFWS_NT_STORE"
variant: $(HDR)
	@mkdir -p $(OBJDIR)/variants/$(V)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) $(F) -Iinclude -Icoldforce_amd/csrc -c coldforce_amd/csrc/cfws_device.hip -o $(OBJDIR)/variants/$(V)/cfws_device.o
	for h in $(HOSTSRC); do $(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) $(F) -Iinclude -Icoldforce_amd/csrc -c coldforce_amd/csrc/$$h.cpp -o $(OBJDIR)/variants/$(V)/$$h.o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OBJDIR)/variants/libcfws_$(V).so $(OBJDIR)/variants/$(V)/*.o

.PHONY: variant
