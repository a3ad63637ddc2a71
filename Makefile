# Build for MI355X (gfx950). Outputs stay in-tree so they travel to the GPU box with gpurun.
#   make            -> oceansimulation_amd/liboceanfft.so (C ABI), libwaves.so (C++ Waves API),
#                      oracle/build/liboceanoracle.so (CPU checker), tests/cpp/test_waves,
#                      examples/waveapp_headless (the reference app's workload, no window)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8

PKG := oceansimulation_amd
CSRC := $(PKG)/csrc
# -fno-slp-vectorize: the SLP vectoriser packs the interleaved float4 arithmetic into v_pk_* with
# shuffles and pushes the column pass past 128 VGPRs (spills). The FFT gets packed math explicitly
# instead (split-plane CPair, ocean_kernels.hip).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fno-slp-vectorize -Wall -Iinclude -I$(CSRC)

LIB := $(PKG)/liboceanfft.so
WAVES := $(PKG)/libwaves.so
ORACLE := oracle/build/liboceanoracle.so
CPPTEST := tests/cpp/test_waves
APP := examples/waveapp_headless

all: $(LIB) $(WAVES) $(ORACLE) $(CPPTEST) $(APP)

DEVICE_H := $(wildcard $(CSRC)/device/*.h) $(CSRC)/ocean_internal.h $(CSRC)/launch_common.h
# one translation unit per frame path, compiled in parallel
KERNEL_TUS := ocean_kernels launch_half launch_slab launch_fft
KERNEL_OBJS := $(KERNEL_TUS:%=$(CSRC)/build/%.o)
$(CSRC)/build/%.o: $(CSRC)/%.hip $(DEVICE_H)
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/build/ocean_capi.o: $(CSRC)/ocean_capi.cpp $(CSRC)/ocean_internal.h include/oceanfft.h
	@mkdir -p $(CSRC)/build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(KERNEL_OBJS) $(CSRC)/build/ocean_capi.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -Wl,-soname,liboceanfft.so -L/opt/rocm/lib -lrccl

# C++ drop-in layer (Waves::FFTCalculator / Waves::Generator / Vision::RenderDevice shim) over the C ABI.
WAVES_SRC := $(CSRC)/waves/RenderDevice.cpp $(CSRC)/waves/FFTCalculator.cpp $(CSRC)/waves/Generator.cpp \
             $(CSRC)/waves/Surface.cpp $(CSRC)/waves/SlabGenerator.cpp
$(WAVES): $(WAVES_SRC) include/waves/Generator.h include/waves/FFTCalculator.h include/waves/Surface.h \
          include/waves/SlabGenerator.h \
          include/vision/RenderDevice.h $(LIB)
	g++ -O2 -std=c++17 -fPIC -shared -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $(WAVES_SRC) \
	    -L$(PKG) -loceanfft -Wl,-rpath,'$$ORIGIN' -L/opt/rocm/lib -lamdhip64

$(ORACLE): oracle/ocean_oracle.c oracle/ocean_oracle.h
	$(MAKE) -s -C oracle

$(CPPTEST): tests/cpp/test_waves.cpp $(WAVES) $(ORACLE)
	g++ -O2 -std=c++17 -Iinclude -Ioracle -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L$(PKG) -lwaves -loceanfft -Loracle/build -loceanoracle \
	    -Wl,-rpath,'$$ORIGIN/../../$(PKG)' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -L/opt/rocm/lib -lamdhip64

# Headless WaveApp (no oracle: its dumps are checked by tests/test_gpu_parity.py)
$(APP): examples/waveapp_headless.cpp $(WAVES)
	g++ -O2 -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L$(PKG) -lwaves -loceanfft -Wl,-rpath,'$$ORIGIN/../$(PKG)' -L/opt/rocm/lib -lamdhip64

MB := tools/microbench
microbench: $(MB)/prebench $(MB)/detbench $(MB)/detbench_soffset $(MB)/rm16bench $(MB)/gen4bench $(MB)/ifft4bench $(MB)/gridbench $(MB)/halfbench_nohs $(MB)/ifftbench $(MB)/transbench $(MB)/scatterbench $(MB)/halfbench $(MB)/genbench $(MB)/colbench $(MB)/copybench $(MB)/genbench_noxch $(MB)/genbench_nobar $(MB)/layoutbench
MB_DEPS := $(KERNEL_TUS:%=$(CSRC)/%.hip) $(DEVICE_H) $(MB)/ab_kernels.h $(MB)/all_kernels.h
$(MB)/%: $(MB)/%.hip $(MB_DEPS)
	$(HIPCC) $(HIPFLAGS) $< -o $@
# timing ablations (wrong results by construction): no LDS exchanges / exchanges without barriers
$(MB)/genbench_noxch: $(MB)/genbench.hip $(MB_DEPS)
	$(HIPCC) $(HIPFLAGS) -DOCEAN_ABLATE_EXCHANGE $< -o $@
$(MB)/halfbench_nohs: $(MB)/halfbench.hip $(MB_DEPS)
	$(HIPCC) $(HIPFLAGS) -DOCEAN_ABLATE_HS $< -o $@
$(MB)/detbench_soffset: $(MB)/detbench.hip $(MB_DEPS)
	$(HIPCC) $(HIPFLAGS) -DOCEAN_SOFFSET_PIECES $< -o $@
$(MB)/genbench_nobar: $(MB)/genbench.hip $(MB_DEPS)
	$(HIPCC) $(HIPFLAGS) -DOCEAN_ABLATE_BARRIER $< -o $@

clean:
	rm -rf $(MB)/detbench $(MB)/detbench_soffset $(MB)/rm16bench $(MB)/gen4bench $(MB)/ifft4bench $(MB)/gridbench $(MB)/halfbench_nohs $(MB)/ifftbench $(MB)/transbench $(MB)/scatterbench $(MB)/halfbench $(MB)/genbench $(MB)/colbench $(MB)/copybench $(MB)/genbench_noxch $(MB)/genbench_nobar $(MB)/layoutbench $(CSRC)/build $(LIB) $(WAVES) $(CPPTEST) $(APP)
	$(MAKE) -s -C oracle clean

.PHONY: all clean microbench
