# Build of the MI355X (gfx950) echo-transform library and its C tools.
#   make            -> xsknet_amd/libxsknet_amd.so (the product), xsknet_amd/libxsknet_amd_tune.so (the product kernel
#                      at alternative switch values, for tools/abbench.py and its parity tests only), oracle/liboracle.so,
#                      tools/echo_replay, tools/rxqueues, tools/rxring
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
CC       := gcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall
CFLAGS   ?= -O2 -std=c11 -Wall -Wextra -fPIC
CSRC     := xsknet_amd/csrc
LIB      := xsknet_amd/libxsknet_amd.so
TUNELIB  := xsknet_amd/libxsknet_amd_tune.so

all: $(LIB) $(TUNELIB) oracle tools/echo_replay tools/rxqueues tools/rxring

# every header a device object or a host object may include (the doorbell layout and host protocol of
# xsk_lowlat_proto.h are shared by xsk_lowlat.hip and xsk_gpu_host.c)
HDRS     := $(CSRC)/xsk_echo_device.h $(CSRC)/xsk_echo_kernels.h $(CSRC)/xsk_hip_util.h $(CSRC)/xsk_gpu_internal.h $(CSRC)/xsk_stage_plan.h \
            $(CSRC)/xsk_lowlat_proto.h $(CSRC)/xsk_ring.h include/xsk_gpu.h
# build id of the transform kernel: a hash of the sources that define it and of the flags, reported by
# xsk_gpu_build_id() so bench.py attaches a PMC traffic summary only to the build it was measured on
# (the device code and its launch: not include/xsk_gpu.h, whose comments change more often than its structs)
BUILD_ID := $(shell cat $(CSRC)/xsk_echo.hip $(CSRC)/xsk_echo_device.h $(CSRC)/xsk_echo_kernels.h $(CSRC)/xsk_hip_util.h | sha256sum | cut -c1-16)-$(shell echo '$(HIPFLAGS)' | sha256sum | cut -c1-4)
HIPOBJ   := $(CSRC)/xsk_echo.o $(CSRC)/xsk_aux.o $(CSRC)/xsk_classify.o $(CSRC)/xsk_lowlat.o
HOSTOBJ  := $(CSRC)/xsk_gpu_host.o $(CSRC)/xsk_gpu_mem.o $(CSRC)/xsk_gpu_rx.o $(CSRC)/xsk_gpu_multi.o $(CSRC)/xsk_gpu_pipe.o $(CSRC)/xsk_gpu_umem.o
TUNEOBJ  := $(CSRC)/tune/xsk_tune_product.o

$(CSRC)/%.o: $(CSRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(CSRC)/xsk_echo.o: $(CSRC)/xsk_echo.hip $(HDRS) Makefile
	$(HIPCC) $(HIPFLAGS) -DXSK_GPU_BUILD_ID='"$(BUILD_ID)"' -c -o $@ $<

$(CSRC)/tune/%.o: $(CSRC)/tune/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(CSRC)/%.o: $(CSRC)/%.c $(HDRS)
	$(CC) $(CFLAGS) -pthread -I$(ROCM)/include -c -o $@ $<

$(LIB): $(HIPOBJ) $(HOSTOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -pthread -Wl,-soname,libxsknet_amd.so

$(TUNELIB): $(TUNEOBJ) $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(TUNEOBJ) -L xsknet_amd -lxsknet_amd \
		-Wl,-rpath,'$$ORIGIN' -Wl,-soname,libxsknet_amd_tune.so

tools/echo_replay: tools/echo_replay.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

tools/rxqueues: tools/rxqueues.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -pthread -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

tools/rxring: tools/rxring.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -pthread -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(CSRC)/*.o $(CSRC)/tune/*.o $(LIB) $(TUNELIB) tools/echo_replay tools/rxqueues tools/rxring
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
