# Build the HIP engine in-tree (the .so travels to the GPU box with the snapshot).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := noisyquantumsimulator_amd
SO := $(PKG)/libryd_engine.so
SRC := $(PKG)/csrc/ryd_engine.hip
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
            -ffp-contract=fast -munsafe-fp-atomics

all: $(SO)

$(SO): $(SRC) $(PKG)/csrc/ryd_traj.inc $(PKG)/csrc/ryd_traj_sym.inc $(PKG)/csrc/ryd_traj_eig.inc $(PKG)/csrc/ryd_traj_wg.inc $(PKG)/csrc/ryd_traj_rows.inc $(PKG)/csrc/ryd_coh_prop.inc $(PKG)/csrc/ryd_dim4_prop.inc $(PKG)/csrc/ryd_shaped16.inc $(PKG)/csrc/ryd_generic.inc $(PKG)/csrc/ryd_sym16.inc $(PKG)/csrc/ryd_epilogue.inc $(PKG)/csrc/ryd_derive.inc include/ryd_engine.h
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC) -ldl

resource-usage: $(SRC)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -o /tmp/ryd_ru.so $(SRC) 2>&1 | \
	  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs:" 

ASM ?= /tmp/ryd_engine.s

asm: $(SRC)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC --cuda-device-only -S -o $(ASM) $(SRC)

# the inline-asm DPP groups: no VALU write within 2 wait states of a DPP read
check-dpp: asm
	python3 tools/check_dpp_hazards.py $(ASM)

clean:
	rm -f $(SO)

.PHONY: all clean resource-usage asm check-dpp
