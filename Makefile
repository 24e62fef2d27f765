# Build of the MI355X (gfx950) echo-transform library and its C tools.
#   make            -> xsknet_amd/libxsknet_amd.so, oracle/liboracle.so, tools/echo_replay
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
CC       := gcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall
CFLAGS   ?= -O2 -std=c11 -Wall -Wextra -fPIC
CSRC     := xsknet_amd/csrc
LIB      := xsknet_amd/libxsknet_amd.so

all: $(LIB) oracle tools/echo_replay

DEVHDR   := $(CSRC)/xsk_echo_device.h $(CSRC)/xsk_echo_variants.h $(CSRC)/xsk_echo_kernels.h $(CSRC)/xsk_hip_util.h include/xsk_gpu.h
HIPOBJ   := $(CSRC)/xsk_echo.o $(CSRC)/xsk_aux.o $(CSRC)/xsk_tune.o $(CSRC)/xsk_classify.o $(CSRC)/xsk_wire.o

$(CSRC)/%.o: $(CSRC)/%.hip $(DEVHDR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(CSRC)/xsk_gpu_host.o: $(CSRC)/xsk_gpu_host.c include/xsk_gpu.h
	$(CC) $(CFLAGS) -I$(ROCM)/include -c -o $@ $<

$(CSRC)/xsk_gpu_rx.o: $(CSRC)/xsk_gpu_rx.c $(CSRC)/xsk_ring.h include/xsk_gpu.h
	$(CC) $(CFLAGS) -c -o $@ $<

$(LIB): $(HIPOBJ) $(CSRC)/xsk_gpu_host.o $(CSRC)/xsk_gpu_rx.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libxsknet_amd.so

tools/echo_replay: tools/echo_replay.c $(LIB) include/xsk_gpu.h
	$(CC) $(CFLAGS) -o $@ $< -L xsknet_amd -lxsknet_amd -Wl,-rpath,'$$ORIGIN/../xsknet_amd'

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(CSRC)/*.o $(LIB) tools/echo_replay
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
