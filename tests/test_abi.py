"""C-ABI boundary checks that need no GPU: the library loads, exports every declared symbol,
and argument validation fails with -EINVAL before touching the device."""
import ctypes as C
import errno
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "xsk_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xsk_gpu_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ("xsk_gpu_echo_dev", "xsk_gpu_init", "xsk_gpu_process", "xsk_gpu_fini", "xsk_gpu_workspace_size",
              "xsk_gpu_ctx_mode",
              "xsk_gpu_synth_dev", "xsk_gpu_rearm_dev", "xsk_gpu_stream_read_dev", "xsk_gpu_abi_version",
              "xsk_gpu_last_error", "xsk_gpu_timing_enable", "xsk_gpu_timing_read"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    import xsknet_amd as X
    L = X.lib()
    for f in declared_functions():
        assert hasattr(L, f), f
    out = subprocess.run(["nm", "-D", "--defined-only", X.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (xsk_gpu_\w+)", out.stdout))
    assert set(declared_functions()) <= exported


def test_struct_layouts_match_header():
    import xsknet_amd as X
    # compile a tiny C probe against the header and compare offsets with the numpy dtypes
    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "xsk_gpu.h"
#define O(s,f) printf(#s "." #f " %zu\n", offsetof(struct s, f))
int main(void){
 printf("desc %zu rec %zu stats %zu\n", sizeof(struct xsk_gpu_desc), sizeof(struct xsk_gpu_rec), sizeof(struct xsk_gpu_stats));
 O(xsk_gpu_rec,verdict);O(xsk_gpu_rec,flags);O(xsk_gpu_rec,ip_proto);O(xsk_gpu_rec,icmp_type);O(xsk_gpu_rec,icmp_code);
 O(xsk_gpu_rec,ip_vihl);O(xsk_gpu_rec,eth_proto);O(xsk_gpu_rec,icmp_csum_in);O(xsk_gpu_rec,icmp_csum_out);
 O(xsk_gpu_rec,ip_sum);O(xsk_gpu_rec,icmp_sum);
 O(xsk_gpu_stats,timestamp);O(xsk_gpu_stats,rx_packets);O(xsk_gpu_stats,rx_bytes);O(xsk_gpu_stats,tx_packets);O(xsk_gpu_stats,tx_bytes);
 O(xsk_gpu_desc,addr);O(xsk_gpu_desc,len);O(xsk_gpu_desc,options);
 return 0;}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "p.c")
        open(c, "w").write(probe)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(td, "p"), c], check=True)
        out = subprocess.run([os.path.join(td, "p")], capture_output=True, text=True, check=True).stdout.split("\n")
    assert out[0] == "desc 16 rec 16 stats 40"
    offs = dict(line.split() for line in out[1:] if line)
    for dt, name in ((X.REC_DTYPE, "xsk_gpu_rec"), (X.STATS_DTYPE, "xsk_gpu_stats"), (X.DESC_DTYPE, "xsk_gpu_desc")):
        for f in dt.names:
            assert int(offs[f"{name}.{f}"]) == dt.fields[f][1], f
    # stats_record (reference xsk_utils.h:17-23) and xdp_desc (linux/if_xdp.h) are the same layouts
    import oracle
    assert oracle.REC_DTYPE == X.REC_DTYPE and oracle.DESC_DTYPE == X.DESC_DTYPE


def test_xdp_desc_binary_compatible():
    probe = r'''
#include <linux/if_xdp.h>
#include <stddef.h>
#include "xsk_gpu.h"
_Static_assert(sizeof(struct xdp_desc) == sizeof(struct xsk_gpu_desc), "size");
_Static_assert(offsetof(struct xdp_desc, len) == offsetof(struct xsk_gpu_desc, len), "len");
_Static_assert(offsetof(struct xdp_desc, options) == offsetof(struct xsk_gpu_desc, options), "opt");
int main(void){return 0;}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "p.c")
        open(c, "w").write(probe)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(td, "p"), c],
                       check=True)


def test_abi_version_and_argument_validation():
    import xsknet_amd as X
    L = X.lib()
    assert L.xsk_gpu_abi_version() == 1
    EINVAL = -errno.EINVAL
    # n == 0 is a no-op that touches nothing
    assert L.xsk_gpu_echo_dev(None, 0, None, 0, None, None, None, None, None) == 0
    # null / misaligned pointers and sizes are rejected before any HIP call
    assert L.xsk_gpu_echo_dev(None, 4096, None, 1, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev(0x1001, 4096, 0x2000, 1, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev(0x1000, 4095, 0x2000, 1, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev(0x1000, 4096, 0x2008, 1, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev(0x1000, 4096, 0x2000, 1, None, 0x3008, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev(0x1000, 4096, 0x2000, 1, None, None, 0x4000, None, None) == EINVAL  # stats w/o ws
    assert L.xsk_gpu_echo_dev(0x1000, 4096, 0x2000, 0xFFFFFFFF, None, None, None, None, None) == EINVAL  # > MAX_BATCH
    # wire-format options: unknown bits and the same argument checks
    assert L.xsk_gpu_echo_dev_opts(0x1000, 4096, 0x2000, 1, 8, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev_opts(0x1001, 4096, 0x2000, 1, 7, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_echo_dev_opts(0x1000, 4096, 0x2000, 0xFFFFFFFF, 7, None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_set_options(None, 1) == EINVAL
    assert L.xsk_gpu_ctx_mode(None) == EINVAL
    assert L.xsk_gpu_synth_dev(0x1000, 1 << 20, 0x2000, 4, 8, 2048, 0, 0, 1, 0, 64, 64, None) == EINVAL
    assert L.xsk_gpu_synth_dev(0x1000, 1 << 20, 0x2000, 4, 0, 32, 0, 0, 1, 0, 64, 64, None) == EINVAL
    assert L.xsk_gpu_synth_dev(0x1000, 1 << 20, 0x2000, 4, 0, 2048, 0, 0, 1, 2, 64, 64, None) == EINVAL
    assert L.xsk_gpu_stream_read_dev(0x1000, 17, 0x2000, None) == EINVAL
    ctx = C.c_void_p()
    import xsknet_amd as X
    buf = X.umem_zeros(4096)
    assert L.xsk_gpu_init(C.byref(ctx), 0, None, 4096, 64, 0) == EINVAL
    # a host UMEM starts on a page of its own (AF_XDP's rule, xsk_utils.c:132-135): 16-B alignment is not enough
    assert L.xsk_gpu_init(C.byref(ctx), 0, buf.ctypes.data + 16, 64, 64, 0) == EINVAL
    assert L.xsk_gpu_init(C.byref(ctx), 0, buf.ctypes.data, 4095, 64, 0) == EINVAL
    assert L.xsk_gpu_init(C.byref(ctx), 0, buf.ctypes.data, 64, 0, 0) == EINVAL
    assert L.xsk_gpu_init(C.byref(ctx), 0, buf.ctypes.data, 64, 64, 7) == EINVAL
    assert L.xsk_gpu_process(None, None, 0, None, None, None) == EINVAL
    L.xsk_gpu_fini(None)


def test_product_library_does_not_link_the_oracle():
    import xsknet_amd as X
    out = subprocess.run(["nm", "-D", X.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "oracle_" not in out
    ldd = subprocess.run(["ldd", X.LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in ldd


def test_kernels_are_gfx950_code_objects():
    """The fat binary embedded in the library carries gfx950 code objects (and only gfx950)."""
    import xsknet_amd as X
    blob = open(X.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob and b"amdgcn-amd-amdhsa--gfx90a" not in blob


def test_tuning_code_is_not_in_the_product_library():
    """Kernel variants and tuning switches live in libxsknet_amd_tune.so only (loaded by tests/tools)."""
    import xsknet_amd as X
    prod = subprocess.run(["nm", "-D", "--defined-only", X.LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    for sym in ("xsk_gpu__product_variant", "timed_round_kernel", "xsk_gpu__echo_variant"):
        assert sym not in prod, sym
    # the product exports the C ABI, plus the CU count the tuning library links against and the test / tool hooks
    # of xsk_gpu_internal.h (LOWLAT diagnostics and knobs, forced grid, multi fault injection and context handles,
    # staged copy-in record and no-alias switch, the UMEM registration references, the kept buffers)
    exported = set(re.findall(r"\bT (\w+)", prod))
    assert exported - set(declared_functions()) <= {"xsk_gpu__num_cu", "xsk_gpu__lowlat_trace", "xsk_gpu__lowlat_tune",
                                                    "xsk_gpu__echo_dev_grid", "xsk_gpu__multi_inject",
                                                    "xsk_gpu__staged_stats", "xsk_gpu__staged_noalias",
                                                    "xsk_gpu__multi_ctx", "xsk_gpu__lowlat_outcomes",
                                                    "xsk_gpu__lowlat_test_width", "xsk_gpu__rx_pipe_ctx",
                                                    "xsk_gpu__lowlat_live", "xsk_gpu__umem_view",
                                                    "xsk_gpu__umem_refs", "xsk_gpu__buf_kept"}, \
        exported - set(declared_functions())
    tune = subprocess.run(["nm", "-D", "--defined-only", X.TUNE_LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    assert "xsk_gpu__product_variant" in tune
    L = X.tune_lib()
    assert hasattr(L, "xsk_gpu__product_variant")
    # the tuning library stays small: the product kernel at a few switch values, no laboratory
    assert os.path.getsize(X.TUNE_LIB_PATH) < 3 << 20


def test_multi_and_lowlat_validation_without_gpu():
    """Argument checks of the multi-context API and the LOWLAT mode constant (no device calls)."""
    import xsknet_amd as X
    L = X.lib()
    EINVAL = -errno.EINVAL
    h = C.c_void_p()
    buf = X.umem_zeros(4096)
    devs = (C.c_int * 1)(0)
    assert L.xsk_gpu_multi_init(C.byref(h), None, 1, buf.ctypes.data, 64, 64, 0) == EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 17, buf.ctypes.data, 64, 64, 0) == EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 1, buf.ctypes.data + 1, 64, 64, 0) == EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 1, buf.ctypes.data + 16, 64, 64, 0) == EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 1, buf.ctypes.data, 64, 0, 0) == EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 1, buf.ctypes.data, 64, 64, 3) == EINVAL
    assert L.xsk_gpu_init(C.byref(h), 0, buf.ctypes.data, 64, 64, 3) == EINVAL
    assert L.xsk_gpu_multi_process(None, None, 0, None, None, None) == EINVAL
    assert L.xsk_gpu_multi_set_options(None, 1) == EINVAL
    # the effective resident-kernel cap is a query: reserving queues lowers it, asking changes nothing
    assert L.xsk_gpu_lowlat_cap(-1) == EINVAL
    c0 = L.xsk_gpu_lowlat_cap(0)
    assert 1 <= c0 <= X.LOWLAT_PER_DEVICE
    assert L.xsk_gpu_lowlat_reserve(0, 1) == c0 - 1 == L.xsk_gpu_lowlat_cap(0) == X.lowlat_cap(0)
    assert L.xsk_gpu_lowlat_reserve(0, 0) == c0 == L.xsk_gpu_lowlat_cap(0)
    L.xsk_gpu_multi_fini(None)
    # the pipelined RX loop: depth 1..XSK_GPU_RX_PIPE_MAX, a valid mode, an aligned UMEM; NULL objects
    assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, buf.ctypes.data, 64, 0, 2) == EINVAL
    assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, buf.ctypes.data, 64, X.RX_PIPE_MAX + 1, 2) == EINVAL
    assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, buf.ctypes.data, 64, 2, 3) == EINVAL
    assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, buf.ctypes.data + 1, 64, 2, 2) == EINVAL
    assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, buf.ctypes.data + 16, 64, 2, 2) == EINVAL
    assert L.xsk_gpu_rx_pipe_init(None, 0, buf.ctypes.data, 64, 2, 2) == EINVAL
    assert L.xsk_gpu_rx_pipe_step(None, None, None, None, None, 64, None, None) == EINVAL
    assert L.xsk_gpu_rx_pipe_flush(None, None, None, None, None) == EINVAL
    assert L.xsk_gpu_rx_pipe_set_options(None, 0) == EINVAL
    assert L.xsk_gpu_rx_pipe_inflight(None) == 0
    L.xsk_gpu_rx_pipe_fini(None)
    hdr = open(HEADER).read()
    assert f"XSK_GPU_RX_PIPE_MAX {X.RX_PIPE_MAX}u" in hdr
    assert "XSK_GPU_MODE_LOWLAT = 2" in hdr and f"XSK_GPU_LOWLAT_MAX {X.LOWLAT_MAX}u" in hdr
    assert f"XSK_GPU_MULTI_MAX {X.MULTI_MAX}" in hdr


def test_product_reads_no_environment():
    """No process-global switch of its own in the product (tuning knobs are explicit entry points of the tools,
    DESIGN.md §1): the only environment variable its sources read is the HIP runtime's GPU_MAX_HW_QUEUES, which bounds
    the resident LOWLAT kernels a device can hold (xsk_gpu_host.c)."""
    import glob
    calls = []
    for p in glob.glob(os.path.join(ROOT, "xsknet_amd", "csrc", "*.[ch]")) + \
            glob.glob(os.path.join(ROOT, "xsknet_amd", "csrc", "*.hip")):
        src = re.sub(r"/\*.*?\*/|//[^\n]*", "", open(p).read(), flags=re.S)
        calls += re.findall(r"\b(?:secure_)?getenv\s*\(([^)]*)\)", src)
    assert calls == ['"GPU_MAX_HW_QUEUES"'], calls


def test_multi_fold_all_or_nothing_c_unit():
    """xsk_gpu_multi_process's counter fold (xsk_gpu__multi_fold, xsk_gpu_internal.h): every share's counters
    when all succeeded, none and the first error when any failed (an injected failing context)."""
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-I", "/opt/rocm/include", "-o", exe,
                        os.path.join(ROOT, "tests", "c", "test_multi_fold.c")], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    assert "multi fold ok" in out


def test_multi_status_validation_without_gpu():
    import xsknet_amd as X
    L = X.lib()
    st = (C.c_int * 4)()
    assert L.xsk_gpu_multi_status(None, st, 4) == -errno.EINVAL


def test_bench_kernel_names_are_the_shipped_kernels():
    """bench.py attributes roofline numbers and PMC summaries to KERNEL / WIRE_KERNEL by rocprofv3's demangled
    name: both must be kernels that libxsknet_amd.so's gfx950 code object really contains."""
    import sys
    from tests.test_lowlat_isa import LLVM, gfx950_code_objects
    import shutil
    filt = shutil.which("c++filt") or (f"{LLVM}/llvm-cxxfilt" if os.path.exists(f"{LLVM}/llvm-cxxfilt") else None)
    if not filt:
        pytest.skip("no demangler (c++filt / llvm-cxxfilt)")
    sys.path.insert(0, ROOT)
    import bench
    import tempfile
    import xsknet_amd as X
    names = set()
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(gfx950_code_objects(X.LIB_PATH)):
            p = os.path.join(td, f"co{k}.o")
            open(p, "wb").write(co)
            syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", p], capture_output=True, text=True,
                                  check=True).stdout
            for line in syms.splitlines():
                f = line.split()
                if len(f) >= 8 and f[3] == "FUNC":
                    names.add(subprocess.run([filt, f[7]], capture_output=True, text=True,
                                             check=True).stdout.strip())
    short = set()
    for nm in names:
        m = re.match(r"^(?:void )?(?:[\w:() ]+::)?(\w+<[^()]*>)\(", nm)
        if m:
            short.add(m.group(1))
    assert bench.KERNEL in short, sorted(short)
    assert bench.WIRE_KERNEL in short, sorted(short)


def test_umem_alloc_without_gpu():
    """xsk_gpu_umem_alloc: 2 MiB aligned, zeroed, writable, argument checks (no device involved)."""
    import xsknet_amd as X
    L = X.lib()
    p = C.c_void_p()
    hb = C.c_uint64(0)
    assert L.xsk_gpu_umem_alloc(C.byref(p), 0, None) == -errno.EINVAL
    assert L.xsk_gpu_umem_alloc(C.byref(p), 4097, None) == -errno.EINVAL
    assert L.xsk_gpu_umem_alloc(None, 4096, None) == -errno.EINVAL
    with X.HugeUmem(5 << 20) as u:
        assert u.array.ctypes.data % (2 << 20) == 0 and u.array.size == 5 << 20
        assert not u.array.any()
        u.array[::4096] = 7
        assert int(u.array.sum()) == 7 * ((5 << 20) // 4096)
        assert 0 <= u.huge_bytes <= 6 << 20
    assert L.xsk_gpu_umem_alloc(C.byref(p), 16 << 20, C.byref(hb)) == 0 and p.value % (2 << 20) == 0
    L.xsk_gpu_umem_free(p, 16 << 20)
    L.xsk_gpu_umem_free(None, 0)
