# Builds the C-ABI library mepol_amd/libmepol_amd.so for gfx950 (MI355X) and the oracle's
# optional C helpers.  `make -j8` here; the .so travels to the GPU box with the snapshot.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
FLAGS   := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
SRC     := $(wildcard mepol_amd/csrc/*.hip)
OBJ     := $(patsubst mepol_amd/csrc/%.hip,build/%.o,$(SRC))
LIB     := mepol_amd/libmepol_amd.so

ORACLE_NATIVE := oracle/native/librollout_kordered.so

all: $(LIB) $(ORACLE_NATIVE)

# the parity oracle's k-ordered rollout (test infrastructure; never linked into the product)
$(ORACLE_NATIVE): oracle/native/rollout_kordered.c
	gcc -O2 -ffp-contract=off -fPIC -shared $< -o $@ -lm

build/%.o: mepol_amd/csrc/%.hip $(wildcard mepol_amd/csrc/*.hpp) include/mepol_amd.h
	@mkdir -p build
	$(HIPCC) $(FLAGS) $(FLAGS_$*) -Iinclude -c $< -o $@

# k-NN selection compares finite MFMA outputs (inputs are validated first): no NaN
# canonicalisation before v_min; MFMA results in VGPRs (no accvgpr copies per tile)
FLAGS_knn := -fno-honor-nans -mllvm -amdgpu-mfma-vgpr-form
FLAGS_knn_select_ks1 := $(FLAGS_knn)
FLAGS_knn_select_ks2 := $(FLAGS_knn)
FLAGS_knn_select_ks3 := $(FLAGS_knn)
FLAGS_knn_select_ks4 := $(FLAGS_knn)

$(LIB): $(OBJ)
	$(HIPCC) $(FLAGS) -shared -o $@ $(OBJ)

resource-usage:
	@for f in $(SRC); do $(HIPCC) $(FLAGS) -Iinclude -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Scratch|Occupancy"; done

clean:
	rm -rf build $(LIB) $(ORACLE_NATIVE)

.PHONY: all clean resource-usage
