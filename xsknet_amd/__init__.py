"""xsknet_amd — MI355X (gfx950) ICMP-echo frame transform behind a C ABI.

The product is ``libxsknet_amd.so`` (HIP kernels + C host code, see ``include/xsk_gpu.h``).  This
module is ctypes plumbing so tests and ``bench.py`` can drive that ABI with torch-allocated device
memory; it contains no compute and has no fallback: if the shared library is missing or cannot be
loaded, importing the bindings raises.

Reference path replaced: ``process_packet``/``csum_replace2`` in
``/root/reference/src/lib/xsk_receive.c:101-190`` called per descriptor from the RX batch loop
``xsk_receive.c:220-233``.
"""
from __future__ import annotations

import ctypes as C
import errno as _errno
import mmap
import os
from typing import Optional

import numpy as np

__all__ = [
    "LIB_PATH", "lib", "build_id", "XskGpuError", "DESC_DTYPE", "REC_DTYPE", "STATS_DTYPE", "VERDICTS",
    "TX_REPLY", "DROP_SHORT", "DROP_NOT_IPV4", "DROP_NOT_ICMP", "DROP_NOT_ECHO", "DROP_BAD_DESC",
    "echo_dev", "synth_dev", "rearm_dev", "stream_read_dev", "workspace_size", "EchoContext",
    "MODE_ZEROCOPY", "MODE_STAGED", "MODE_LOWLAT", "LOWLAT_MAX", "MultiContext", "tune_lib", "lowlat_reserve", "lowlat_cap", "timing_enable", "timing_read", "Ring", "FramePool", "RxResult",
    "classify_dev", "XDP_DROP", "XDP_PASS", "XDP_REDIRECT", "DROP_BAD_IP", "DROP_BAD_CSUM",
    "OPT_STRICT_IPV4", "OPT_VLAN", "OPT_VERIFY_CSUM", "OPT_ALL", "F_IP_CSUM_OK", "F_ICMP_CSUM_OK", "F_VLAN",
    "F_IP_OPTIONS",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libxsknet_amd.so")
# the product kernel at alternative switch values for in-process A/B (tools/abbench.py) and its parity tests; never
# the product path
TUNE_LIB_PATH = os.path.join(_HERE, "libxsknet_amd_tune.so")

TX_REPLY, DROP_SHORT, DROP_NOT_IPV4, DROP_NOT_ICMP, DROP_NOT_ECHO, DROP_BAD_DESC, DROP_BAD_IP, DROP_BAD_CSUM = range(8)
VERDICTS = ["TX_REPLY", "DROP_SHORT", "DROP_NOT_IPV4", "DROP_NOT_ICMP", "DROP_NOT_ECHO", "DROP_BAD_DESC",
            "DROP_BAD_IP", "DROP_BAD_CSUM"]
# wire-format options (include/xsk_gpu.h XSK_GPU_OPT_*) and record flags
OPT_STRICT_IPV4, OPT_VLAN, OPT_VERIFY_CSUM, OPT_ALL = 1, 2, 4, 7
F_IP_CSUM_OK, F_ICMP_CSUM_OK, F_VLAN, F_IP_OPTIONS = 1, 2, 4, 8
MODE_ZEROCOPY, MODE_STAGED, MODE_LOWLAT = 0, 1, 2
LOWLAT_MAX = 1024  # XSK_GPU_LOWLAT_MAX
RX_PIPE_MAX = 8  # XSK_GPU_RX_PIPE_MAX
MULTI_MAX = 16  # XSK_GPU_MULTI_MAX
LOWLAT_PER_DEVICE = 8  # XSK_GPU_LOWLAT_PER_DEVICE (the cap is min(this, GPU_MAX_HW_QUEUES), 4 by default)

# struct xsk_gpu_desc == struct xdp_desc (linux/if_xdp.h)
DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
# struct xsk_gpu_rec (16 B)
REC_DTYPE = np.dtype([
    ("verdict", "u1"), ("flags", "u1"), ("ip_proto", "u1"), ("icmp_type", "u1"),
    ("icmp_code", "u1"), ("ip_vihl", "u1"), ("eth_proto", "<u2"), ("icmp_csum_in", "<u2"),
    ("icmp_csum_out", "<u2"), ("ip_sum", "<u2"), ("icmp_sum", "<u2"),
])
# struct xsk_gpu_stats == struct stats_record (xsk_utils.h:17-23)
STATS_DTYPE = np.dtype([("timestamp", "<u8"), ("rx_packets", "<u8"), ("rx_bytes", "<u8"),
                        ("tx_packets", "<u8"), ("tx_bytes", "<u8")])
assert DESC_DTYPE.itemsize == 16 and REC_DTYPE.itemsize == 16 and STATS_DTYPE.itemsize == 40


class XskGpuError(RuntimeError):
    def __init__(self, fn: str, rc: int):
        name = _errno.errorcode.get(-rc, str(rc))
        detail = ""
        if _lib is not None:
            detail = f" (last HIP error: {_lib.xsk_gpu_last_error().decode()})"
        super().__init__(f"{fn} failed: -{name}{detail}")
        self.rc = rc


class Ring(C.Structure):
    """struct xsk_gpu_ring == libxdp's struct xsk_ring_prod / xsk_ring_cons."""
    _fields_ = [("cached_prod", C.c_uint32), ("cached_cons", C.c_uint32), ("mask", C.c_uint32),
                ("size", C.c_uint32), ("producer", C.c_void_p), ("consumer", C.c_void_p), ("ring", C.c_void_p),
                ("flags", C.c_void_p)]


class FramePool(C.Structure):
    """struct xsk_gpu_frame_pool: the client's free-frame stack (xsk_utils.h:30-31)."""
    _fields_ = [("addr", C.c_void_p), ("n_free", C.c_uint32), ("capacity", C.c_uint32)]


class RxResult(C.Structure):
    _fields_ = [("received", C.c_uint32), ("replied", C.c_uint32), ("tx_full", C.c_uint32),
                ("refilled", C.c_uint32)]


assert C.sizeof(Ring) == 48 and C.sizeof(FramePool) == 16 and C.sizeof(RxResult) == 16

_lib: Optional[C.CDLL] = None

_P = C.c_void_p
_SIGS = {
    "xsk_gpu_abi_version": ([], C.c_int),
    "xsk_gpu_last_error": ([], C.c_char_p),
    "xsk_gpu_build_id": ([], C.c_char_p),
    "xsk_gpu_workspace_size": ([C.c_int, C.c_uint32], C.c_size_t),
    "xsk_gpu_echo_dev": ([_P, C.c_uint64, _P, C.c_uint32, _P, _P, _P, _P, _P], C.c_int),
    "xsk_gpu_echo_dev_opts": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P], C.c_int),
    "xsk_gpu_set_options": ([_P, C.c_uint32], C.c_int),
    "xsk_gpu_init": ([C.POINTER(_P), C.c_int, _P, C.c_uint64, C.c_uint32, C.c_int], C.c_int),
    "xsk_gpu_process": ([_P, _P, C.c_uint32, _P, _P, _P], C.c_int),
    "xsk_gpu_fini": ([_P], None),
    "xsk_gpu_ctx_mode": ([_P], C.c_int),
    "xsk_gpu_synth_dev": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                           C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, _P], C.c_int),
    "xsk_gpu_rearm_dev": ([_P, _P, _P, C.c_uint32, _P], C.c_int),
    "xsk_gpu_stream_read_dev": ([_P, C.c_uint64, _P, _P], C.c_int),
    "xsk_gpu_timing_enable": ([C.c_int], C.c_int),
    "xsk_gpu_timing_read": ([C.POINTER(C.c_double), C.POINTER(C.c_uint64)], C.c_int),
    "xsk_gpu_rx_step": ([_P, C.POINTER(Ring), C.POINTER(Ring), C.POINTER(Ring), C.POINTER(FramePool), C.c_uint32,
                         _P, C.POINTER(RxResult)], C.c_int),
    "xsk_gpu_tx_complete": ([C.POINTER(Ring), C.POINTER(FramePool), C.c_uint32], C.c_uint32),
    "xsk_gpu_classify_workspace_size": ([C.c_uint32], C.c_size_t),
    "xsk_gpu_classify_dev": ([_P, C.c_uint64, _P, C.c_uint32, C.c_int, _P, _P, _P, _P, _P], C.c_int),
    "xsk_gpu_multi_init": ([C.POINTER(_P), _P, C.c_uint32, _P, C.c_uint64, C.c_uint32, C.c_int], C.c_int),
    "xsk_gpu_multi_process": ([_P, _P, C.c_uint32, _P, _P, _P], C.c_int),
    "xsk_gpu_multi_set_options": ([_P, C.c_uint32], C.c_int),
    "xsk_gpu_multi_status": ([_P, _P, C.c_uint32], C.c_int),
    "xsk_gpu_stats_tx_failed": ([_P, _P, _P, _P, C.c_uint32], C.c_int),
    "xsk_gpu__multi_inject": ([_P, C.c_uint32, C.c_int], C.c_int),
    "xsk_gpu__lowlat_tune": ([_P, C.c_uint32, C.c_uint32, C.c_uint32], C.c_int),
    "xsk_gpu_multi_fini": ([_P], None),
    "xsk_gpu_lowlat_reserve": ([C.c_int, C.c_uint32], C.c_int),
    "xsk_gpu_lowlat_cap": ([C.c_int], C.c_int),
    "xsk_gpu__umem_refs": ([_P], C.c_int),
    "xsk_gpu__buf_kept": ([C.c_int], C.c_int),
    "xsk_gpu__staged_stats": ([_P, C.POINTER(C.c_uint64)], C.c_int),
    "xsk_gpu__staged_noalias": ([_P, C.c_uint32], C.c_int),
    "xsk_gpu__lowlat_outcomes": ([_P, C.POINTER(C.c_uint64)], C.c_int),
    "xsk_gpu__lowlat_test_width": ([_P, C.c_uint32], C.c_int),
    "xsk_gpu__multi_ctx": ([_P, C.c_uint32], _P),
    "xsk_gpu__lowlat_live": ([C.c_int, C.POINTER(C.c_uint32)], C.c_int),
    "xsk_gpu__umem_view": ([_P, C.c_uint64, _P, C.c_uint64], C.c_int),
    "xsk_gpu_umem_alloc": ([C.POINTER(_P), C.c_uint64, C.POINTER(C.c_uint64)], C.c_int),
    "xsk_gpu_umem_free": ([_P, C.c_uint64], None),
    "xsk_gpu_rx_pipe_init": ([C.POINTER(_P), C.c_int, _P, C.c_uint64, C.c_uint32, C.c_int], C.c_int),
    "xsk_gpu_rx_pipe_step": ([_P, C.POINTER(Ring), C.POINTER(Ring), C.POINTER(Ring), C.POINTER(FramePool), C.c_uint32,
                              _P, C.POINTER(RxResult)], C.c_int),
    "xsk_gpu_rx_pipe_flush": ([_P, C.POINTER(Ring), C.POINTER(FramePool), _P, C.POINTER(RxResult)], C.c_int),
    "xsk_gpu_rx_pipe_set_options": ([_P, C.c_uint32], C.c_int),
    "xsk_gpu_rx_pipe_inflight": ([_P], C.c_uint32),
    "xsk_gpu_rx_pipe_depth": ([_P], C.c_uint32),
    "xsk_gpu_rx_pipe_fini": ([_P], None),
    "xsk_gpu__rx_pipe_ctx": ([_P, C.c_uint32], _P),
    # internal test / tool hook (xsk_gpu_internal.h): the product kernel with a forced workgroup count
    "xsk_gpu__echo_dev_grid": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint32], C.c_int),
}
_TUNE_SIGS = {
    "xsk_gpu__product_variant": ([C.c_int, C.c_uint32, _P, C.c_uint64, _P, C.c_uint32, _P, _P, _P, _P], C.c_int),
}
_tune: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load libxsknet_amd.so (raises OSError if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def tune_lib() -> C.CDLL:
    """libxsknet_amd_tune.so: the product kernel at alternative switch values (tools/abbench.py, tests only)."""
    global _tune
    if _tune is None:
        lib()
        if not os.path.exists(TUNE_LIB_PATH):
            raise OSError(f"{TUNE_LIB_PATH} not built: run `make`")
        L = C.CDLL(TUNE_LIB_PATH)
        for name, (args, res) in _TUNE_SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _tune = L
    return _tune


def _check(fn: str, rc: int) -> None:
    if rc != 0:
        raise XskGpuError(fn, rc)


def _ptr(t) -> Optional[int]:
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return t.data_ptr()


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


def build_id() -> str:
    """xsk_gpu_build_id(): hash of the transform kernel's sources and flags in the loaded library."""
    return lib().xsk_gpu_build_id().decode()


def workspace_size(device: int, n: int) -> int:
    return int(lib().xsk_gpu_workspace_size(device, n))


def echo_dev(umem, descs, n: int, verdicts=None, recs=None, stats=None, workspace=None, stream=None,
             opts: int = 0, grid: int = 0) -> None:
    """xsk_gpu_echo_dev (opts == 0) / xsk_gpu_echo_dev_opts on torch device tensors (uint8 umem,
    uint8/int64 views of the structs).  grid != 0: the same product kernel with that many workgroups for a
    large batch (internal hook xsk_gpu__echo_dev_grid, tests only)."""
    if grid:
        _check("xsk_gpu__echo_dev_grid", lib().xsk_gpu__echo_dev_grid(
            _ptr(umem), umem.numel() * umem.element_size(), _ptr(descs), n, opts, _ptr(verdicts), _ptr(recs),
            _ptr(stats), _ptr(workspace), _stream_ptr(stream), grid))
        return
    if opts:
        _check("xsk_gpu_echo_dev_opts", lib().xsk_gpu_echo_dev_opts(
            _ptr(umem), umem.numel() * umem.element_size(), _ptr(descs), n, opts, _ptr(verdicts), _ptr(recs),
            _ptr(stats), _ptr(workspace), _stream_ptr(stream)))
        return
    _check("xsk_gpu_echo_dev", lib().xsk_gpu_echo_dev(
        _ptr(umem), umem.numel() * umem.element_size(), _ptr(descs), n, _ptr(verdicts), _ptr(recs), _ptr(stats),
        _ptr(workspace), _stream_ptr(stream)))


XDP_DROP, XDP_PASS, XDP_REDIRECT = 1, 2, 4


def classify_dev(umem, descs, n: int, bound: bool, actions, out=None, nout=None, workspace=None, stream=None) -> None:
    """xsk_gpu_classify_dev: the XDP ingress filter (inner_xdp.c:26-61) + in-order compaction."""
    if workspace is None:
        import torch
        workspace = torch.empty(int(lib().xsk_gpu_classify_workspace_size(max(n, 1))), dtype=torch.uint8,
                                device=umem.device)
    _check("xsk_gpu_classify_dev", lib().xsk_gpu_classify_dev(
        _ptr(umem), umem.numel() * umem.element_size(), _ptr(descs), n, 1 if bound else 0, _ptr(actions), _ptr(out),
        _ptr(nout), _ptr(workspace), _stream_ptr(stream)))


def synth_dev(umem, descs, n: int, base_off: int, stride: int, seed: int, first: int = 0, step: int = 1,
              mode: int = 0, len_lo: int = 1500, len_hi: int = 1500, stream=None) -> None:
    _check("xsk_gpu_synth_dev", lib().xsk_gpu_synth_dev(
        _ptr(umem), umem.numel() * umem.element_size(), _ptr(descs), n, base_off, stride, seed, first, step, mode,
        len_lo, len_hi, _stream_ptr(stream)))


def rearm_dev(umem, descs, verdicts, n: int, stream=None) -> None:
    _check("xsk_gpu_rearm_dev", lib().xsk_gpu_rearm_dev(_ptr(umem), _ptr(descs), _ptr(verdicts), n,
                                                        _stream_ptr(stream)))


def stream_read_dev(src, nbytes: int, out, stream=None) -> None:
    _check("xsk_gpu_stream_read_dev", lib().xsk_gpu_stream_read_dev(_ptr(src), nbytes, _ptr(out),
                                                                    _stream_ptr(stream)))


def lowlat_reserve(device: int, queues: int) -> int:
    """xsk_gpu_lowlat_reserve: set aside highest-priority hardware queues of `device` for the application's own
    highest-priority streams; returns the resident LOWLAT kernels now allowed there."""
    rc = lib().xsk_gpu_lowlat_reserve(device, queues)
    if rc < 0:
        raise XskGpuError("xsk_gpu_lowlat_reserve", rc)
    return rc



def lowlat_cap(device: int = 0) -> int:
    """xsk_gpu_lowlat_cap: the resident LOWLAT kernels this process may run on `device` now (min(8,
    GPU_MAX_HW_QUEUES) less the reserved queues), without changing anything."""
    rc = lib().xsk_gpu_lowlat_cap(device)
    if rc < 0:
        raise XskGpuError("xsk_gpu_lowlat_cap", rc)
    return rc

def timing_enable(on: bool = True) -> None:
    _check("xsk_gpu_timing_enable", lib().xsk_gpu_timing_enable(1 if on else 0))


def timing_read():
    ms = C.c_double(0.0)
    cnt = C.c_uint64(0)
    _check("xsk_gpu_timing_read", lib().xsk_gpu_timing_read(C.byref(ms), C.byref(cnt)))
    return ms.value, cnt.value


def lowlat_live(device: int = 0) -> int:
    """Workgroups of resident LOWLAT grids running on `device` in this process (xsk_gpu__lowlat_live)."""
    out = C.c_uint32(0)
    _check("xsk_gpu__lowlat_live", lib().xsk_gpu__lowlat_live(device, C.byref(out)))
    return int(out.value)


def umem_zeros(nbytes: int) -> np.ndarray:
    """A zeroed host UMEM on pages of its own: an anonymous mapping, so its base is page-aligned as xsk_gpu_init /
    xsk_gpu_multi_init / xsk_gpu_rx_pipe_init require and AF_XDP does -- the counterpart of the reference's
    posix_memalign(getpagesize(), ...) (src/lib/xsk_utils.c:132-135).  A plain numpy array is not: its data may start
    inside a page another allocation shares."""
    nbytes = int(nbytes)
    return np.frombuffer(mmap.mmap(-1, max(nbytes, 1)), np.uint8, count=nbytes)


def umem_copy(a: np.ndarray) -> np.ndarray:
    """umem_zeros of a's size holding a's bytes."""
    out = umem_zeros(a.nbytes)
    out[:] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    return out


class HugeUmem:
    """xsk_gpu_umem_alloc / xsk_gpu_umem_free: a UMEM on transparent huge pages (2 MiB aligned, touched up front);
    `.array` is its numpy uint8 view, `.huge_bytes` how much of it the kernel backed with huge pages."""

    def __init__(self, size: int):
        self._p = C.c_void_p()
        hb = C.c_uint64(0)
        _check("xsk_gpu_umem_alloc", lib().xsk_gpu_umem_alloc(C.byref(self._p), size, C.byref(hb)))
        self.size = size
        self.huge_bytes = int(hb.value)
        self.array = np.ctypeslib.as_array((C.c_uint8 * size).from_address(self._p.value))

    def close(self) -> None:
        if self._p:
            self.array = None
            lib().xsk_gpu_umem_free(self._p, self.size)
            self._p = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


STAGED_FIELDS = ("h2d_bytes", "strided", "span", "gather", "contained", "hostpack", "own_dma")


def staged_stats_of(ctx) -> dict:
    """xsk_gpu__staged_stats of a STAGED context handle: bytes copied host->device since init (frame bytes, plus the
    host pack's 4-B staging offsets), the chunks copied as one 2-D stride / one dense span / by the gather kernel, the
    chunks whose copy-in wrote only their own frames' mirror bytes (run without waiting for the previous chunk's header
    pack), the chunks copied by the host pack (no mapped alias), and the frames of those too large for a staging half
    (a DMA copy each)."""
    out = (C.c_uint64 * len(STAGED_FIELDS))()
    _check("xsk_gpu__staged_stats", lib().xsk_gpu__staged_stats(ctx, out))
    return dict(zip(STAGED_FIELDS, (int(x) for x in out)))


class EchoContext:
    """Host-UMEM drop-in (xsk_gpu_init / xsk_gpu_process / xsk_gpu_fini) over a numpy uint8 UMEM."""

    def __init__(self, umem: np.ndarray, device: int = 0, max_batch: int = 4096, mode: int = MODE_ZEROCOPY,
                 opts: int = 0):
        assert umem.dtype == np.uint8 and umem.flags.c_contiguous
        self.umem = umem
        self._ctx = C.c_void_p()
        _check("xsk_gpu_init", lib().xsk_gpu_init(C.byref(self._ctx), device, umem.ctypes.data, umem.nbytes,
                                                  max_batch, mode))
        if opts:
            self.set_options(opts)

    def set_options(self, opts: int) -> None:
        _check("xsk_gpu_set_options", lib().xsk_gpu_set_options(self._ctx, opts))

    @property
    def mode(self) -> int:
        """xsk_gpu_ctx_mode: the mode the context runs in (a LOWLAT request beyond XSK_GPU_LOWLAT_PER_DEVICE on its
        device runs as ZEROCOPY)."""
        return lib().xsk_gpu_ctx_mode(self._ctx)

    def process(self, descs: np.ndarray, want_recs: bool = True):
        n = len(descs)
        descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
        verdicts = np.zeros(n, np.uint8)
        recs = np.zeros(n, REC_DTYPE) if want_recs else None
        stats = np.zeros(1, STATS_DTYPE)
        _check("xsk_gpu_process", lib().xsk_gpu_process(
            self._ctx, descs.ctypes.data, n, verdicts.ctypes.data, recs.ctypes.data if recs is not None else None,
            stats.ctypes.data))
        return verdicts, recs, stats[0]

    def staged_stats(self):
        """xsk_gpu__staged_stats of a STAGED context (see staged_stats_of)."""
        return staged_stats_of(self._ctx)

    def drop_alias(self, half_bytes: int = 0) -> None:
        """Test switch (xsk_gpu__staged_noalias): the STAGED context forgets its UMEM's mapped device alias, as on a
        device where the runtime gives none, so its scattered copy-ins take the host pack (staging halves of
        half_bytes; 0 = the default 32 MiB)."""
        _check("xsk_gpu__staged_noalias", lib().xsk_gpu__staged_noalias(self._ctx, half_bytes))

    def lowlat_tune(self, tile_frames: int = 0, groups: int = 0, timeout_us: int = 0) -> None:
        """Tool / test knobs of a LOWLAT context (xsk_gpu__lowlat_tune): frames per wave, serving workgroups,
        completion timeout (0 = defaults)."""
        _check("xsk_gpu__lowlat_tune", lib().xsk_gpu__lowlat_tune(self._ctx, tile_frames, groups, timeout_us))

    def lowlat_test_width(self, wgs: int) -> None:
        """Test switch (xsk_gpu__lowlat_test_width): launch the resident grid with `wgs` workgroups (0 = all)."""
        _check("xsk_gpu__lowlat_test_width", lib().xsk_gpu__lowlat_test_width(self._ctx, wgs))

    def umem_view(self, off: int, n: int) -> np.ndarray:
        """xsk_gpu__umem_view: n bytes at `off` as the GPU's translation of the UMEM sees them (ZEROCOPY / LOWLAT)."""
        out = np.zeros(n, np.uint8)
        _check("xsk_gpu__umem_view", lib().xsk_gpu__umem_view(self._ctx, off, out.ctypes.data, n))
        return out

    def lowlat_outcomes(self):
        """xsk_gpu__lowlat_outcomes: doorbell batches that missed their timeout -- all, completed through the launch
        path after a partial service, returned -ETIMEDOUT, completed late (every slice served, found after STOP)."""
        out = (C.c_uint64 * 4)()
        _check("xsk_gpu__lowlat_outcomes", lib().xsk_gpu__lowlat_outcomes(self._ctx, out))
        return {"timeouts": int(out[0]), "partial": int(out[1]), "untouched": int(out[2]), "late": int(out[3])}

    def rx_step(self, rx: Ring, fill: Ring, tx: Ring, pool: FramePool, max_batch: int, stats=None):
        """xsk_gpu_rx_step on this context; returns (received, RxResult)."""
        res = RxResult()
        rc = lib().xsk_gpu_rx_step(self._ctx, C.byref(rx), C.byref(fill), C.byref(tx), C.byref(pool), max_batch,
                                   stats.ctypes.data if stats is not None else None, C.byref(res))
        if rc < 0:
            raise XskGpuError("xsk_gpu_rx_step", rc)
        return rc, res

    def close(self) -> None:
        if self._ctx:
            lib().xsk_gpu_fini(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiContext:
    """xsk_gpu_multi_*: one host UMEM, one context per entry of ``devices`` (repeats allowed), descriptor i
    of a batch on context i mod G, counters summed."""

    def __init__(self, umem: np.ndarray, devices, max_batch: int = 4096, mode: int = MODE_ZEROCOPY, opts: int = 0):
        assert umem.dtype == np.uint8 and umem.flags.c_contiguous
        self.umem = umem
        self._ctx = C.c_void_p()
        devs = (C.c_int * len(devices))(*devices)
        _check("xsk_gpu_multi_init", lib().xsk_gpu_multi_init(C.byref(self._ctx), devs, len(devices), umem.ctypes.data,
                                                              umem.nbytes, max_batch, mode))
        if opts:
            _check("xsk_gpu_multi_set_options", lib().xsk_gpu_multi_set_options(self._ctx, opts))

    def process(self, descs: np.ndarray, want_recs: bool = True):
        n = len(descs)
        descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
        verdicts = np.zeros(n, np.uint8)
        recs = np.zeros(n, REC_DTYPE) if want_recs else None
        stats = np.zeros(1, STATS_DTYPE)
        _check("xsk_gpu_multi_process", lib().xsk_gpu_multi_process(
            self._ctx, descs.ctypes.data, n, verdicts.ctypes.data, recs.ctypes.data if recs is not None else None,
            stats.ctypes.data))
        return verdicts, recs, stats[0]

    def status(self):
        """xsk_gpu_multi_status: per-context result of the last process() (0 or -errno)."""
        st = (C.c_int * MULTI_MAX)()
        g = lib().xsk_gpu_multi_status(self._ctx, st, MULTI_MAX)
        if g < 0:
            raise XskGpuError("xsk_gpu_multi_status", g)
        return list(st[:g])

    def context(self, g: int):
        """Context g's handle (xsk_gpu__multi_ctx), for staged_stats_of."""
        h = lib().xsk_gpu__multi_ctx(self._ctx, g)
        if not h:
            raise XskGpuError("xsk_gpu__multi_ctx", -22)
        return h

    def staged_stats(self):
        """Every context's xsk_gpu__staged_stats (STAGED mode), in context order."""
        return [staged_stats_of(self.context(g)) for g in range(len(self.status()))]

    def drop_alias(self, half_bytes: int = 0) -> None:
        """Test switch: every context forgets the UMEM's mapped alias (xsk_gpu__staged_noalias)."""
        for g in range(len(self.status())):
            _check("xsk_gpu__staged_noalias", lib().xsk_gpu__staged_noalias(self.context(g), half_bytes))

    def inject_failure(self, g: int, rc: int) -> None:
        """Test hook: context g's next share fails with rc (xsk_gpu__multi_inject)."""
        _check("xsk_gpu__multi_inject", lib().xsk_gpu__multi_inject(self._ctx, g, rc))

    def close(self) -> None:
        if self._ctx:
            lib().xsk_gpu_multi_fini(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ContextView(EchoContext):
    """A context owned by another object (a pipelined RX loop's): EchoContext's queries and test knobs, no ownership."""

    def __init__(self, handle):  # noqa: super().__init__ is not called: nothing is created
        self.umem = None
        self._ctx = C.c_void_p(handle)

    def close(self) -> None:
        self._ctx = C.c_void_p()


class RxPipe:
    """xsk_gpu_rx_pipe_*: the RX loop step with up to ``depth`` batches in flight, one per context of ``mode`` over one
    registration of the UMEM (include/xsk_gpu.h)."""

    def __init__(self, umem: np.ndarray, device: int = 0, depth: int = 2, mode: int = MODE_LOWLAT, opts: int = 0):
        assert umem.dtype == np.uint8 and umem.flags.c_contiguous
        self.umem = umem
        self.depth_asked = depth
        self._p = C.c_void_p()
        _check("xsk_gpu_rx_pipe_init", lib().xsk_gpu_rx_pipe_init(C.byref(self._p), device, umem.ctypes.data,
                                                                  umem.nbytes, depth, mode))
        if opts:
            self.set_options(opts)

    def set_options(self, opts: int) -> None:
        _check("xsk_gpu_rx_pipe_set_options", lib().xsk_gpu_rx_pipe_set_options(self._p, opts))

    def step(self, rx: Ring, fill: Ring, tx: Ring, pool: FramePool, max_batch: int, stats=None):
        """xsk_gpu_rx_pipe_step: returns (frames completed, RxResult)."""
        res = RxResult()
        rc = lib().xsk_gpu_rx_pipe_step(self._p, C.byref(rx), C.byref(fill), C.byref(tx), C.byref(pool), max_batch,
                                        stats.ctypes.data if stats is not None else None, C.byref(res))
        if rc < 0:
            raise XskGpuError("xsk_gpu_rx_pipe_step", rc)
        return rc, res

    def flush(self, tx: Ring, pool: FramePool, stats=None):
        """xsk_gpu_rx_pipe_flush: returns (frames completed, RxResult)."""
        res = RxResult()
        rc = lib().xsk_gpu_rx_pipe_flush(self._p, C.byref(tx), C.byref(pool),
                                         stats.ctypes.data if stats is not None else None, C.byref(res))
        if rc < 0:
            raise XskGpuError("xsk_gpu_rx_pipe_flush", rc)
        return rc, res

    @property
    def inflight(self) -> int:
        return int(lib().xsk_gpu_rx_pipe_inflight(self._p))

    @property
    def depth(self) -> int:
        """Contexts the pipe holds: a LOWLAT pipe keeps doorbell contexts only (xsk_gpu_rx_pipe_depth)."""
        return int(lib().xsk_gpu_rx_pipe_depth(self._p))

    def context(self, i: int) -> ContextView:
        """Context i of the pipe (xsk_gpu__rx_pipe_ctx): its mode, LOWLAT knobs and outcomes."""
        h = lib().xsk_gpu__rx_pipe_ctx(self._p, i)
        if not h:
            raise XskGpuError("xsk_gpu__rx_pipe_ctx", -22)
        return ContextView(h)

    def close(self) -> None:
        if self._p:
            lib().xsk_gpu_rx_pipe_fini(self._p)
            self._p = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
