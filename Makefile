# Build of the MI355X (gfx950) echo-transform library and its C tools.
#   make            -> xsknet_amd/libxsknet_amd.so (the product), xsknet_amd/libxsknet_amd_tune.so (kernel
#                      variants for tools/kbench.py and their parity tests only), oracle/liboracle.so,
#                      tools/echo_replay
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
CC       := gcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall
CFLAGS   ?= -O2 -std=c11 -Wall -Wextra -fPIC
CSRC     := xsknet_amd/csrc
LIB      := xsknet_amd/libxsknet_amd.so
TUNELIB  := xsknet_amd/libxsknet_amd_tune.so

all: $(LIB) $(TUNELIB) oracle tools/echo_replay tools/rxqueues

DEVHDR   := $(CSRC)/xsk_echo_device.h $(CSRC)/xsk_echo_kernels.h $(CSRC)/xsk_hip_util.h include/xsk_gpu.h
# build id of the transform kernel: a hash of the sources that define it and of the flags, reported by
# xsk_gpu_build_id() so bench.py attaches a PMC traffic summary only to the build it was measured on
# (the device code and its launch: not include/xsk_gpu.h, whose comments change more often than its structs)
BUILD_ID := $(shell cat $(CSRC)/xsk_echo.hip $(CSRC)/xsk_echo_device.h $(CSRC)/xsk_echo_kernels.h $(CSRC)/xsk_hip_util.h | sha256sum | cut -c1-16)-$(shell echo '$(HIPFLAGS)' | sha256sum | cut -c1-4)
HIPOBJ   := $(CSRC)/xsk_echo.o $(CSRC)/xsk_aux.o $(CSRC)/xsk_classify.o $(CSRC)/xsk_lowlat.o
HOSTOBJ  := $(CSRC)/xsk_gpu_host.o $(CSRC)/xsk_gpu_rx.o $(CSRC)/xsk_gpu_multi.o
TUNEOBJ  := $(CSRC)/tune/xsk_tune.o $(CSRC)/tune/xsk_wire_v1.o $(CSRC)/tune/xsk_tune_product.o $(CSRC)/tune/xsk_tune_slack.o

$(CSRC)/%.o: $(CSRC)/%.hip $(DEVHDR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(CSRC)/xsk_echo.o: $(CSRC)/xsk_echo.hip $(DEVHDR) Makefile
	$(HIPCC) $(HIPFLAGS) -DXSK_GPU_BUILD_ID='"$(BUILD_ID)"' -c -o $@ $<

$(CSRC)/tune/%.o: $(CSRC)/tune/%.hip $(DEVHDR) $(CSRC)/tune/xsk_echo_variants.h $(CSRC)/tune/xsk_echo_lab.h
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(CSRC)/%.o: $(CSRC)/%.c include/xsk_gpu.h $(CSRC)/xsk_gpu_internal.h $(CSRC)/xsk_ring.h
	$(CC) $(CFLAGS) -pthread -I$(ROCM)/include -c -o $@ $<

# the round-4 candidate SLACK, on a copy of the product header (tune/xsk_tune_slack.hip)
$(CSRC)/xsk_echo_device_slack.gen.h: $(CSRC)/xsk_echo_device.h tools/slack_header.patch
	patch -s -o $@ $(CSRC)/xsk_echo_device.h tools/slack_header.patch

$(CSRC)/tune/xsk_tune_slack.o: $(CSRC)/tune/xsk_tune_slack.hip $(CSRC)/xsk_echo_device_slack.gen.h $(DEVHDR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(HIPOBJ) $(HOSTOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -pthread -Wl,-soname,libxsknet_amd.so

$(TUNELIB): $(TUNEOBJ) $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(TUNEOBJ) -L xsknet_amd -lxsknet_amd \
		-Wl,-rpath,'$$ORIGIN' -Wl,-soname,libxsknet_amd_tune.so

tools/echo_replay: tools/echo_replay.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

tools/rxqueues: tools/rxqueues.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -pthread -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(CSRC)/*.o $(CSRC)/tune/*.o $(LIB) $(TUNELIB) tools/echo_replay tools/rxqueues $(CSRC)/xsk_echo_device_slack.gen.h
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
