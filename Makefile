# Build of every native artefact (hipcc cross-compiles gfx950 without a GPU).
#   make            -> library + drivers + oracle
#   make lib        -> spmm_amd/lib/libmi355_spgemm.so  (the product)
#   make drivers    -> drivers/bin/spgemm_from_txt_alg{1,2,3}
#   make oracle     -> oracle/liboracle.so              (test infrastructure)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Wall
LIB      := spmm_amd/lib/libmi355_spgemm.so
SRC      := spmm_amd/csrc/spgemm.hip
HDRS     := include/spgemm.h $(wildcard spmm_amd/csrc/*.hpp)
DRIVERS  := drivers/bin/spgemm_from_txt_alg1 drivers/bin/spgemm_from_txt_alg2 drivers/bin/spgemm_from_txt_alg3

FASTPATH := spmm_amd/lib/fastpath/spmm_fastpath.so

all: lib drivers oracle fastpath
lib: $(LIB)
drivers: $(DRIVERS)
fastpath: $(FASTPATH)

# torch C++ extension of the Python shim (links the library above; no device code)
$(FASTPATH): spmm_amd/csrc/fastpath.cpp include/spgemm.h spmm_amd/build_fastpath.py $(LIB)
	python3 spmm_amd/build_fastpath.py

# the source id (sources + effective HIPFLAGS) is compiled into the library: spg_build_info()
$(LIB): $(SRC) $(HDRS) spmm_amd/source_id.py
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSPG_SOURCE_ID='"$(shell python3 spmm_amd/source_id.py '$(HIPFLAGS)')"' \
	    -DSPG_HIPFLAGS='"$(strip $(HIPFLAGS))"' -shared -Wl,-soname,libmi355_spgemm.so -Iinclude -Ispmm_amd/csrc \
	    $(SRC) -o $@

# the three reference driver names, one source; ALG fixed at compile time
drivers/bin/spgemm_from_txt_alg%: drivers/spgemm_from_txt.cpp include/spgemm.h $(LIB)
	@mkdir -p $(dir $@)
	g++ -O2 -std=c++17 -Wall -DSPG_DRIVER_ALG=$* -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
	    $< -o $@ -L$(abspath spmm_amd/lib) -lmi355_spgemm -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../spmm_amd/lib' -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle liboracle.so

clean:
	rm -f $(LIB) $(DRIVERS)
	rm -rf spmm_amd/lib/fastpath
	$(MAKE) -s -C oracle clean

.PHONY: all lib drivers oracle fastpath clean
