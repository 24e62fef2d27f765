// xsk_hip_util.h — error plumbing shared by the C-ABI translation units (host code).
#pragma once

#include <errno.h>
#include <hip/hip_runtime.h>

// Records hipGetErrorName(e) for xsk_gpu_last_error() and maps e to a negative errno.
extern "C" __attribute__((visibility("hidden"))) int xsk_gpu__hip_fail(hipError_t e);

#define HIP_TRY(expr)                                           \
    do {                                                        \
        const hipError_t e__ = (expr);                          \
        if (e__ != hipSuccess) return xsk_gpu__hip_fail(e__);   \
    } while (0)
