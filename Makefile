# Native build of the seed-extension engine (gfx950 only) and its test infrastructure.
#   make            -> product library + tools + oracle
#   make product    -> bwa-mem2-arm_amd/lib/libbsw_hip.so   (HIP kernels + C ABI)
#   make oracle     -> oracle/liboracle.so                  (CPU oracle + SSE4.1 baseline; tests only)
PKG      := bwa-mem2-arm_amd
CSRC     := $(PKG)/csrc
LIBDIR   := $(PKG)/lib
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function \
            -munsafe-fp-atomics -Iinclude
CFLAGS   ?= -O3 -fPIC -Wall -Iinclude

PRODUCT  := $(LIBDIR)/libbsw_hip.so
SYNTH    := $(LIBDIR)/libbsw_synth.so
SHIMTEST := $(LIBDIR)/bsw_shim_example
ORACLE   := oracle/liboracle.so

HIP_SRCS := $(CSRC)/bsw_kernels.hip $(CSRC)/bsw_pc.hip $(CSRC)/bsw_wv.hip $(CSRC)/bsw_gq.hip $(CSRC)/bsw_mate.hip $(CSRC)/bsw_global.hip $(CSRC)/bsw_ext_dev.hip $(CSRC)/bsw_fmi.hip $(CSRC)/bsw_fmi_build.hip $(CSRC)/bsw_memchain.hip $(CSRC)/bsw_chain.hip $(CSRC)/bsw_host.cpp $(CSRC)/bsw_ext.cpp $(CSRC)/bsw_pack.cpp $(CSRC)/bsw_devcache.cpp
HIP_HDRS := $(CSRC)/bsw_devcache.h $(CSRC)/bsw_pool.h $(CSRC)/bsw_kernels.h $(CSRC)/bsw_mate_k.h include/bsw_mate.h $(CSRC)/bsw_global_k.h include/bsw_global.h $(CSRC)/bsw_ext_k.h $(CSRC)/bsw_wave.h $(CSRC)/bsw_internal.h $(CSRC)/bsw_fmi_internal.h include/bsw.h include/bsw_seqpair.h include/bsw_ext.h include/bsw_batch.h include/bsw_fmi.h

all: product synth oracle percall

PERCALL := $(LIBDIR)/percall_bench
percall: $(PERCALL)
$(PERCALL): tools/percall_bench.cpp $(PRODUCT) $(SYNTH) include/bsw.h
	g++ -O2 -std=c++17 -pthread -Iinclude -o $@ $< $(PRODUCT) $(SYNTH) -Wl,-rpath,'$$ORIGIN'

product: $(PRODUCT)
synth: $(SYNTH)
oracle: $(ORACLE)

$(LIBDIR):
	mkdir -p $(LIBDIR)

$(LIBDIR)/bsw_kernels.o: $(CSRC)/bsw_kernels.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_pc.o: $(CSRC)/bsw_pc.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_wv.o: $(CSRC)/bsw_wv.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_gq.o: $(CSRC)/bsw_gq.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_mate.o: $(CSRC)/bsw_mate.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_global.o: $(CSRC)/bsw_global.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_ext_dev.o: $(CSRC)/bsw_ext_dev.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_fmi.o: $(CSRC)/bsw_fmi.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_chain.o: $(CSRC)/bsw_chain.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_memchain.o: $(CSRC)/bsw_memchain.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_fmi_build.o: $(CSRC)/bsw_fmi_build.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_host.o: $(CSRC)/bsw_host.cpp $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIBDIR)/bsw_ext.o: $(CSRC)/bsw_ext.cpp $(HIP_HDRS) | $(LIBDIR)
	g++ -O3 -std=c++17 -fPIC -Wall -Iinclude -c $< -o $@

$(LIBDIR)/bsw_pack.o: $(CSRC)/bsw_pack.cpp $(CSRC)/bsw_internal.h | $(LIBDIR)
	g++ -O3 -std=c++17 -fPIC -Wall -Iinclude -c $< -o $@

$(LIBDIR)/bsw_devcache.o: $(CSRC)/bsw_devcache.cpp $(CSRC)/bsw_devcache.h | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/bsw_batch.o: $(CSRC)/bsw_batch.c include/bsw_batch.h include/bsw.h | $(LIBDIR)
	gcc $(CFLAGS) -std=c11 -c $< -o $@

$(PRODUCT): $(LIBDIR)/bsw_kernels.o $(LIBDIR)/bsw_pc.o $(LIBDIR)/bsw_wv.o $(LIBDIR)/bsw_gq.o $(LIBDIR)/bsw_mate.o $(LIBDIR)/bsw_global.o $(LIBDIR)/bsw_ext_dev.o $(LIBDIR)/bsw_fmi.o $(LIBDIR)/bsw_fmi_build.o $(LIBDIR)/bsw_memchain.o $(LIBDIR)/bsw_chain.o $(LIBDIR)/bsw_host.o $(LIBDIR)/bsw_ext.o $(LIBDIR)/bsw_pack.o $(LIBDIR)/bsw_devcache.o $(LIBDIR)/bsw_batch.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

$(SYNTH): $(CSRC)/bsw_synth.c include/bsw_seqpair.h | $(LIBDIR)
	gcc $(CFLAGS) -shared -o $@ $<

ORACLE_SRCS := oracle/ksw_ext_ref.c oracle/bsw_sse41.c oracle/bsw_avx512.c oracle/ext_ref.c oracle/ksw_align_ref.c oracle/ksw_global_ref.c oracle/fmi_ref.c oracle/chain_ref.c
$(ORACLE): $(ORACLE_SRCS) oracle/bsw_simd_batch.inc oracle/bsw_simd_common.h include/bsw_seqpair.h include/bsw_ext.h include/bsw_fmi.h
	gcc $(CFLAGS) -msse4.1 -shared -o $@ $(ORACLE_SRCS) -lpthread

clean:
	rm -f $(LIBDIR)/*.o $(LIBDIR)/*.so $(ORACLE)

# experiment build: pc_kernel group-path counters (tools/pc_stats.py), never loaded by the product
STATSLIB := $(LIBDIR)/libbsw_hip_stats.so
stats: $(STATSLIB)
$(LIBDIR)/bsw_pc_stats.o: $(CSRC)/bsw_pc.hip $(HIP_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DBSW_PC_STATS -c $< -o $@
$(STATSLIB): $(LIBDIR)/bsw_kernels.o $(LIBDIR)/bsw_pc_stats.o $(LIBDIR)/bsw_wv.o $(LIBDIR)/bsw_gq.o $(LIBDIR)/bsw_mate.o $(LIBDIR)/bsw_global.o $(LIBDIR)/bsw_ext_dev.o $(LIBDIR)/bsw_fmi.o $(LIBDIR)/bsw_fmi_build.o $(LIBDIR)/bsw_memchain.o $(LIBDIR)/bsw_chain.o $(LIBDIR)/bsw_host.o $(LIBDIR)/bsw_ext.o $(LIBDIR)/bsw_pack.o $(LIBDIR)/bsw_devcache.o $(LIBDIR)/bsw_batch.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

# experiment build: the product with bsw_pc.hip compiled under AB_FLAGS (same-box A/B runs: tools/ab_lib.sh)
ABLIB := $(LIBDIR)/libbsw_hip_ab.so
AB_FLAGS ?=
ab:
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $(CSRC)/bsw_pc.hip -o $(LIBDIR)/bsw_pc_ab.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(ABLIB) $(LIBDIR)/bsw_kernels.o $(LIBDIR)/bsw_pc_ab.o $(LIBDIR)/bsw_wv.o $(LIBDIR)/bsw_gq.o $(LIBDIR)/bsw_mate.o $(LIBDIR)/bsw_global.o $(LIBDIR)/bsw_ext_dev.o $(LIBDIR)/bsw_fmi.o $(LIBDIR)/bsw_fmi_build.o $(LIBDIR)/bsw_memchain.o $(LIBDIR)/bsw_chain.o $(LIBDIR)/bsw_host.o $(LIBDIR)/bsw_ext.o $(LIBDIR)/bsw_pack.o $(LIBDIR)/bsw_devcache.o $(LIBDIR)/bsw_batch.o -lpthread

# the same for bsw_host.cpp (host pipeline experiments): libbsw_hip_abhost.so
ABHOSTLIB := $(LIBDIR)/libbsw_hip_abhost.so
abhost:
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -x hip -c $(CSRC)/bsw_host.cpp -o $(LIBDIR)/bsw_host_ab.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(ABHOSTLIB) $(LIBDIR)/bsw_kernels.o $(LIBDIR)/bsw_pc.o $(LIBDIR)/bsw_wv.o $(LIBDIR)/bsw_gq.o $(LIBDIR)/bsw_mate.o $(LIBDIR)/bsw_global.o $(LIBDIR)/bsw_ext_dev.o $(LIBDIR)/bsw_fmi.o $(LIBDIR)/bsw_fmi_build.o $(LIBDIR)/bsw_memchain.o $(LIBDIR)/bsw_chain.o $(LIBDIR)/bsw_host_ab.o $(LIBDIR)/bsw_ext.o $(LIBDIR)/bsw_pack.o $(LIBDIR)/bsw_devcache.o $(LIBDIR)/bsw_batch.o -lpthread

# the same for bsw_fmi.hip (SMEM walk experiments): libbsw_hip_abfmi.so
ABFMILIB := $(LIBDIR)/libbsw_hip_abfmi.so
abfmi:
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $(CSRC)/bsw_fmi.hip -o $(LIBDIR)/bsw_fmi_ab.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(ABFMILIB) $(LIBDIR)/bsw_kernels.o $(LIBDIR)/bsw_pc.o $(LIBDIR)/bsw_wv.o $(LIBDIR)/bsw_gq.o $(LIBDIR)/bsw_mate.o $(LIBDIR)/bsw_global.o $(LIBDIR)/bsw_ext_dev.o $(LIBDIR)/bsw_fmi_ab.o $(LIBDIR)/bsw_fmi_build.o $(LIBDIR)/bsw_memchain.o $(LIBDIR)/bsw_chain.o $(LIBDIR)/bsw_host.o $(LIBDIR)/bsw_ext.o $(LIBDIR)/bsw_pack.o $(LIBDIR)/bsw_devcache.o $(LIBDIR)/bsw_batch.o -lpthread

.PHONY: all product synth oracle percall clean stats ab abfmi abhost

# host sanitizer build: AddressSanitizer + UBSan over the host C / C++ of the
# product (bsw_pack.cpp, bsw_ext.cpp, bsw_batch.c, bsw_synth.c) and the oracle, driven by
# tools/asan/asan_driver.cpp with an oracle-backed engine stub (no GPU).  Log: tools/asan/asan.log
ASAN_DIR   := tools/asan
ASAN_FLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g -O1 -Iinclude
ASAN_BIN   := $(ASAN_DIR)/asan_driver
ASAN_C     := $(CSRC)/bsw_batch.c $(CSRC)/bsw_synth.c oracle/ksw_ext_ref.c oracle/ext_ref.c oracle/ksw_align_ref.c oracle/ksw_global_ref.c oracle/fmi_ref.c oracle/chain_ref.c
ASAN_SSE   := oracle/bsw_sse41.c oracle/bsw_avx512.c
ASAN_CXX   := $(ASAN_DIR)/asan_driver.cpp $(ASAN_DIR)/engine_stub.cpp $(CSRC)/bsw_ext.cpp $(CSRC)/bsw_pack.cpp
$(ASAN_BIN): $(ASAN_C) $(ASAN_SSE) oracle/bsw_simd_batch.inc oracle/bsw_simd_common.h $(ASAN_CXX) $(CSRC)/bsw_internal.h include/bsw_ext.h include/bsw_fmi.h
	mkdir -p $(ASAN_DIR)/obj
	for f in $(ASAN_C); do gcc $(ASAN_FLAGS) -std=gnu11 -c $$f -o $(ASAN_DIR)/obj/$$(basename $$f).o || exit 1; done
	for f in $(ASAN_SSE); do gcc $(ASAN_FLAGS) -std=gnu11 -msse4.1 -c $$f -o $(ASAN_DIR)/obj/$$(basename $$f).o || exit 1; done
	g++ $(ASAN_FLAGS) -std=c++17 -o $@ $(ASAN_CXX) $(ASAN_DIR)/obj/*.o -lpthread
asan: $(ASAN_BIN)
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	  ./$(ASAN_BIN) > $(ASAN_DIR)/asan.log 2>&1; rc=$$?; cat $(ASAN_DIR)/asan.log; exit $$rc
# the CPU test suite (-m "not gpu") against sanitized builds of the oracle and the synthetic
# generator (LD_PRELOAD of the sanitizer runtimes into python; leak checks off: the interpreter
# keeps its arenas).  Log: tools/asan/asan_suite.log
ASAN_ORACLE := $(ASAN_DIR)/liboracle_asan.so
ASAN_SYNTH  := $(ASAN_DIR)/libbsw_synth_asan.so
$(ASAN_ORACLE): $(ORACLE_SRCS) oracle/bsw_simd_batch.inc oracle/bsw_simd_common.h include/bsw_seqpair.h include/bsw_ext.h include/bsw_fmi.h
	mkdir -p $(ASAN_DIR)
	gcc $(ASAN_FLAGS) -fPIC -msse4.1 -shared -o $@ $(ORACLE_SRCS) -lpthread
$(ASAN_SYNTH): $(CSRC)/bsw_synth.c include/bsw_seqpair.h
	mkdir -p $(ASAN_DIR)
	gcc $(ASAN_FLAGS) -fPIC -shared -o $@ $(CSRC)/bsw_synth.c
asan-suite: $(ASAN_ORACLE) $(ASAN_SYNTH)
	LD_PRELOAD="$$(gcc -print-file-name=libasan.so) $$(gcc -print-file-name=libubsan.so)" \
	  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	  BSW_ORACLE_LIB=$(ASAN_ORACLE) BSW_SYNTH_LIB=$(ASAN_SYNTH) \
	  python -m pytest tests -q -m "not gpu" -p no:cacheprovider > $(ASAN_DIR)/asan_suite.log 2>&1; rc=$$?; \
	  tail -5 $(ASAN_DIR)/asan_suite.log; exit $$rc
.PHONY: asan asan-suite
