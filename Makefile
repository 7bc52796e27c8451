# Build: product library (gfx950 HIP + host C++), oracle (plain C, test
# infrastructure), C++ parity test.  No cmake: hipcc / gcc directly.
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
CXX     ?= g++
ARCH    ?= gfx950
BUILD   := build

INC      := -Iinclude -Icyclone_amd/csrc
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result $(INC)
HOSTFLAGS:= -O2 -std=c++17 -fPIC -Wall $(INC) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include

LIB      := cyclone_amd/libcyaes.so
MGPU     := cyclone_amd/libcyaes_mgpu.so
ORACLE   := oracle/liboracle.so
CPPTEST  := $(BUILD)/test_rijndael $(BUILD)/relay_calls
# Measurement-only build of the same kernels with the in-kernel clock probe
# (CYAES_CLOCK_PROBE): bench.py reads the shader clock under load from it.
PROBE    := $(BUILD)/variants/clockprobe.so
# Bounds-checked build of the same kernels (CYAES_BOUNDS_CHECK): every global
# access checked against its batch-contract extent, misses counted (never
# faulted) and read by cyaes_debug_bounds(); the GPU suite runs on it with
# CYAES_LIBRARY=build/variants/bounds.so.
BOUNDS   := $(BUILD)/variants/bounds.so

# AES kernels in three translation units, each compiled with the machine
# scheduler that measured best for its kernels (profiles/r03/ab_sched.txt):
# the default for the quad encrypt and the ragged decrypt, iterative ILP for
# the lane encrypt (config C -1.5 %), max ILP for the flat decrypt (-1.5 %).
KSRC     := cyclone_amd/csrc/cyaes_kernels.hip
ESRC     := cyclone_amd/csrc/cyaes_enc_kernels.hip
DSRC     := cyclone_amd/csrc/cyaes_dec_kernels.hip
XSRC     := cyclone_amd/csrc/cyaes_duplex_kernels.hip
RSRC     := cyclone_amd/csrc/cyaes_ragged_kernels.hip
SCHED_ENC:= -mllvm -amdgpu-sched-strategy=iterative-ilp
SCHED_DEC:= -mllvm -amdgpu-sched-strategy=max-ilp
SCHED_K  ?=
SCHED_RAG?= -mllvm -amdgpu-sched-strategy=iterative-ilp
ASRC     := cyclone_amd/csrc/cyaes_adler.hip
BSRC     := cyclone_amd/csrc/cyaes_batch_kernels.hip
HSRC     := cyclone_amd/csrc/cyaes_runtime.cpp cyclone_amd/csrc/cyaes_pins.cpp cyclone_amd/csrc/cyaes_tables.cpp cyclone_amd/csrc/cyr_rijndael.cpp \
            cyclone_amd/csrc/cyaes_relay.cpp cyclone_amd/csrc/cyaes_batcher.cpp
HDRS     := include/cyaes.h include/cyaes_relay.h include/cyaes_batch.h include/cyclone_amd/cyr_rijndael.h cyclone_amd/csrc/cyaes_internal.h \
            cyclone_amd/csrc/cyaes_tables.h
KHDRS    := $(HDRS) cyclone_amd/csrc/cyaes_device.h cyclone_amd/csrc/cyaes_enc_body.h cyclone_amd/csrc/cyaes_dec_body.h \
            cyclone_amd/csrc/cyaes_lines_body.h

KOBJ     := $(BUILD)/cyaes_kernels.o $(BUILD)/cyaes_enc_kernels.o $(BUILD)/cyaes_dec_kernels.o $(BUILD)/cyaes_duplex_kernels.o \
            $(BUILD)/cyaes_ragged_kernels.o
AOBJ     := $(BUILD)/cyaes_adler.o
BOBJ     := $(BUILD)/cyaes_batch_kernels.o
HOBJ     := $(patsubst cyclone_amd/csrc/%.cpp,$(BUILD)/%.o,$(HSRC))

.PHONY: all lib mgpu oracle cpptest probe bounds microbench variant clean
all: lib mgpu oracle cpptest probe bounds $(BUILD)/bench_batcher $(BUILD)/relay_loop $(BUILD)/dropin_threads $(BUILD)/hostlink
lib: $(LIB)
mgpu: $(MGPU)
oracle: $(ORACLE)
cpptest: $(CPPTEST)
probe: $(PROBE)
bounds: $(BOUNDS)

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/cyaes_kernels.o: $(KSRC) $(KHDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SCHED_K) -c $< -o $@

$(BUILD)/cyaes_enc_kernels.o: $(ESRC) $(KHDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SCHED_ENC) -c $< -o $@

$(BUILD)/cyaes_dec_kernels.o: $(DSRC) $(KHDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SCHED_DEC) -c $< -o $@

# The duplex kernel holds both walks; one scheduler for the translation unit
# (SCHED_DUPLEX): iterative ILP, under which both walks compile to the hot
# blocks of their own translation units or better (encrypt 3,659 instructions /
# 168 s_waitcnt per chunk as k_encrypt; decrypt 1,749 / 12 per step against
# k_decrypt_flat's 1,790 / 53); under max ILP the encrypt walk fell to 642 waits.
SCHED_DUPLEX ?= $(SCHED_ENC)
$(BUILD)/cyaes_duplex_kernels.o: $(XSRC) $(KHDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SCHED_DUPLEX) -c $< -o $@

# The ragged decrypt (r05): iterative ILP (profiles/r05/ab_ragged_sched.txt)
$(BUILD)/cyaes_ragged_kernels.o: $(RSRC) $(KHDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(SCHED_RAG) -c $< -o $@

# The kernel objects of a variant build: $(call kvariant,NAME,DEFS)
define kvariant
	mkdir -p $(BUILD)/variants
	$(HIPCC) $(HIPFLAGS) $(SCHED_K) $(2) -c $(KSRC) -o $(BUILD)/variants/$(1).o
	$(HIPCC) $(HIPFLAGS) $(SCHED_ENC) $(2) -c $(ESRC) -o $(BUILD)/variants/$(1)_enc.o
	$(HIPCC) $(HIPFLAGS) $(SCHED_DEC) $(2) -c $(DSRC) -o $(BUILD)/variants/$(1)_dec.o
	$(HIPCC) $(HIPFLAGS) $(SCHED_DUPLEX) $(2) -c $(XSRC) -o $(BUILD)/variants/$(1)_dup.o
	$(HIPCC) $(HIPFLAGS) $(SCHED_RAG) $(2) -c $(RSRC) -o $(BUILD)/variants/$(1)_rag.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(BUILD)/variants/$(1).so $(BUILD)/variants/$(1).o \
	  $(BUILD)/variants/$(1)_enc.o $(BUILD)/variants/$(1)_dec.o $(BUILD)/variants/$(1)_dup.o $(BUILD)/variants/$(1)_rag.o \
	  $(AOBJ) $(BOBJ) $(HOBJ)
endef

$(AOBJ): $(ASRC) include/cyaes_adler32.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BOBJ): $(BSRC) $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: cyclone_amd/csrc/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(KOBJ) $(AOBJ) $(BOBJ) $(HOBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

# Single-process multi-GPU front end: separate library so libcyaes.so does not pull in RCCL.
$(MGPU): cyclone_amd/csrc/cyaes_mgpu.cpp include/cyaes_mgpu.h $(LIB)
	$(HIPCC) $(HOSTFLAGS) -shared -o $@ $< -Lcyclone_amd -lcyaes -L/opt/rocm/lib -lrccl -Wl,-rpath,'$$ORIGIN'

$(ORACLE): oracle/aes_oracle.c
	$(CC) -O2 -fPIC -shared -pthread -Wall -o $@ $<

$(BUILD)/test_rijndael: tests/cpp/test_rijndael.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) -O2 -std=c++17 -Wall $(INC) -o $@ $< -Lcyclone_amd -lcyaes -Wl,-rpath,'$$ORIGIN/../cyclone_amd'

# The relay's Rijndael call expressions, verbatim; -DNDEBUG as a release build
$(BUILD)/relay_calls: tests/cpp/relay_calls.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) -O2 -DNDEBUG -std=c++17 -Wall -Wno-misleading-indentation $(INC) -o $@ $< -Lcyclone_amd -lcyaes -Wl,-rpath,'$$ORIGIN/../cyclone_amd'

microbench: $(BUILD)/microbench $(BUILD)/bench_batcher

$(BUILD)/bench_batcher: tools/bench_batcher.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) -O2 -std=c++17 -Wall -pthread $(INC) -o $@ $< -Lcyclone_amd -lcyaes -Wl,-rpath,'$$ORIGIN/../cyclone_amd'

$(BUILD)/dropin_threads: tools/dropin_threads.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) -O2 -std=c++17 -Wall -pthread $(INC) -o $@ $< -Lcyclone_amd -lcyaes -Wl,-rpath,'$$ORIGIN/../cyclone_amd'

# Kernel-driven host<->HBM packet moves vs DMA (the batcher's zero-copy gather/scatter)
$(BUILD)/hostlink: tools/hostlink.hip | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -o $@ $<

$(BUILD)/microbench: tools/microbench.hip | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -o $@ $<

$(PROBE): $(KSRC) $(ESRC) $(DSRC) $(XSRC) $(RSRC) $(KHDRS) $(HOBJ) $(AOBJ) $(BOBJ)
	$(call kvariant,clockprobe,-DCYAES_CLOCK_PROBE=1)

$(BOUNDS): $(KSRC) $(ESRC) $(DSRC) $(XSRC) $(RSRC) $(KHDRS) $(HOBJ) $(AOBJ) $(BOBJ)
	$(call kvariant,bounds,-DCYAES_BOUNDS_CHECK=1)

# A/B variants: make variant NAME=x DEFS="-DFOO=1" -> build/variants/x.so
variant: $(HOBJ) $(AOBJ) $(BOBJ) | $(BUILD)
	$(call kvariant,$(NAME),$(DEFS))

clean:
	rm -rf $(BUILD) $(LIB) $(MGPU) $(ORACLE)

# The relay's whole data path through the batching adapter (SEAL, tunnel stream, parse, OPEN), one process
$(BUILD)/relay_loop: tools/relay_loop.cpp $(LIB) $(HDRS) | $(BUILD)
	$(CXX) -O2 -std=c++17 -Wall -pthread $(INC) -o $@ $< -Lcyclone_amd -lcyaes -Wl,-rpath,'$$ORIGIN/../cyclone_amd'
