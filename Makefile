# Build the MI355X library (HIP, gfx950) and the CPU oracle (test infrastructure).
#   make            -> real_time_ray_tracer_amd/librtrt.so, oracle/build/librt_oracle.so, build/rt_headless
#   make lib|oracle|headless|clean
#   make ablib      -> build/librtrt_ab.so: the same shim over tools/ab/rt_kernels_ab.hip, the launcher
#                      with the experimental A/B kernels and their RTRT_* environment switches
#                      (tools/ab.py: RTRT_LIB=build/librtrt_ab.so); never part of librtrt.so
HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
ARCH     ?= gfx950
PKG      := real_time_ray_tracer_amd
CSRC     := $(PKG)/csrc
OBJDIR   := build/obj

# -ffp-contract=off + correctly-rounded f32 '/' and sqrt: the float semantics shared with the
# oracle (oracle/rt_oracle.h).  No fast-math anywhere.
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off $(HIPFLAGS_EXTRA) \
            -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -Wall -Wno-unused-function -Iinclude
CFLAGS_ORACLE := -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp -fPIC -std=c99 -Wall

LIB      := $(PKG)/librtrt.so
ORACLE   := oracle/build/librt_oracle.so
ORACLE_NATIVE := oracle/build/librt_oracle_zen.so
HEADLESS := build/rt_headless

all: lib oracle headless
lib: $(LIB)
oracle: $(ORACLE) $(ORACLE_NATIVE)
headless: $(HEADLESS)

# kernels whose leading arguments are scalars (hybrid_kernel's tables, selftest_kernel) get
# them preloaded into SGPRs at wave launch (gfx950 kernarg preload; FrameParams is never preloaded)
KARG_PRELOAD ?= -mllvm -amdgpu-kernarg-preload-count=7

$(OBJDIR)/rt_kernels.o: $(CSRC)/rt_kernels.hip $(CSRC)/*.h include/rt/*.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(KARG_PRELOAD) -x hip -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.hip $(CSRC)/*.h include/rt/*.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/rt_host.o: $(CSRC)/rt_host.cpp include/rt/*.h | $(OBJDIR)
	$(HIPCC) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Iinclude -c $< -o $@

$(OBJDIR)/rt_group.o: $(CSRC)/rt_group.cpp include/rt/*.h | $(OBJDIR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Iinclude -c $< -o $@

# BUILD_INFO: sha1 of the library's sources (+ the git commit they were built at, "+dirty" if
# they differ from it), so measurements can name the kernel code they were taken on
$(LIB): $(OBJDIR)/rt_kernels.o $(OBJDIR)/rt_shim.o $(OBJDIR)/rt_host.o $(OBJDIR)/rt_group.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread
	@src=$$(cat $(CSRC)/*.hip $(CSRC)/*.h $(CSRC)/rt_host.cpp $(CSRC)/rt_group.cpp include/rt/*.h Makefile | sha1sum | cut -c1-12); \
	 commit=$$(git rev-parse --short=12 HEAD 2>/dev/null || echo unknown); \
	 git diff --quiet HEAD -- $(CSRC) include Makefile 2>/dev/null || commit="$$commit+dirty"; \
	 printf '{"src_sha1": "%s", "commit": "%s"}\n' "$$src" "$$commit" > $(dir $@)BUILD_INFO

ABLIB := build/librtrt_ab.so
$(OBJDIR)/rt_kernels_ab.o: tools/ab/rt_kernels_ab.hip $(CSRC)/*.h include/rt/*.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(KARG_PRELOAD) -I$(CSRC) -x hip -c $< -o $@

$(ABLIB): $(OBJDIR)/rt_kernels_ab.o $(OBJDIR)/rt_shim.o $(OBJDIR)/rt_host.o $(OBJDIR)/rt_group.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

ablib: $(ABLIB)

# A compile-time variant of the production library for tools/ab.py --libs (same sources, extra
# defines):  make variant V=post32x8 VFLAGS="-DRT_POST_BWX=4 -DRT_POST_BWY=1"  -> build/v_post32x8/librtrt.so
variant:
	$(MAKE) lib OBJDIR=build/v_$(V)/obj LIB=build/v_$(V)/librtrt.so HIPFLAGS_EXTRA="$(VFLAGS)"

$(ORACLE): oracle/rt_oracle.c oracle/rt_oracle.h include/rt/layout.h
	@mkdir -p oracle/build
	$(CC) $(CFLAGS_ORACLE) -shared -o $@ oracle/rt_oracle.c -lquadmath -lm

# CPU-baseline build for the GPU box's AMD EPYC (Zen 5) host cores; same source and float flags
$(ORACLE_NATIVE): oracle/rt_oracle.c oracle/rt_oracle.h include/rt/layout.h
	@mkdir -p oracle/build
	$(CC) $(subst -march=x86-64-v3,-march=znver3 -mtune=znver3 -mavx512f -mavx512cd -mavx512bw -mavx512dq -mavx512vl,$(CFLAGS_ORACLE)) -shared -o $@ oracle/rt_oracle.c -lquadmath -lm

$(HEADLESS): $(CSRC)/rt_headless.cpp $(LIB) include/rt/*.h
	$(CXX) -O2 -std=c++17 -Iinclude -o $@ $< -L$(PKG) -lrtrt -Wl,-rpath,'$$ORIGIN/../$(PKG)'

$(OBJDIR):
	@mkdir -p $(OBJDIR)

clean:
	rm -rf build oracle/build $(LIB)

.PHONY: all lib oracle headless ablib variant clean
