// Shared device/host helpers for the gtsfm_amd HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

#include "gtsfm_hip.h"

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define GTSFM_CHECK_HIP(expr)                          \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return GTSFM_ERR_HIP;    \
    } while (0)

// Raises a kernel's dynamic-LDS limit to `bytes` on the CURRENT device, once per (kernel, device) and size;
// thread-safe (the attribute is per device, so a process-global "done" flag would skip the second GPU).
static inline hipError_t gtsfm_set_dynamic_lds(const void* fn, int bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    int& have = done[{fn, dev}];
    if (have >= bytes) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) have = bytes;
    return e;
}

__host__ __device__ static inline size_t gtsfm_align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Lane-wise min/max/median of three unsigned keys (v_min_u32 / v_med3_u32).
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;  // one v_med3_u32 (the generic min/max form is not always matched by the backend)
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;  // one v_min3_u32
    asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Insert two keys a, b into a running (b1 <= b2) top-2: 3 ops instead of 4. The second smallest of
// {b1, b2, a, b} is min(b2, med3(b1, a, b)) because b2 >= b1.
__device__ __forceinline__ void top2_insert2(uint32_t& b1, uint32_t& b2, uint32_t a, uint32_t b) {
    const uint32_t m = umed3(b1, a, b);
    b1 = umin3(b1, a, b);
    b2 = umin(b2, m);
}

// (a << s) | b in one v_lshl_or_b32 (keeps the backend from splitting shared shifts into shift + or pairs)
__device__ __forceinline__ uint32_t lshl_or(uint32_t a, uint32_t s, uint32_t b) {
    uint32_t r;
    asm volatile("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(b));
    return r;
}

// Insert key k into a running (b1 <= b2) top-2 of packed keys: second = med3(b1, b2, k), first = min(b1, k).
__device__ __forceinline__ void top2_insert(uint32_t& b1, uint32_t& b2, uint32_t k) {
    b2 = umed3(b1, b2, k);
    b1 = umin(b1, k);
}

// Merge two top-2 lists (a1 <= a2, c1 <= c2) into a.
__device__ __forceinline__ void top2_merge(uint32_t& a1, uint32_t& a2, uint32_t c1, uint32_t c2) {
    uint32_t n1 = umin(a1, c1);
    uint32_t n2 = umin(umax(a1, c1), umin(a2, c2));
    a1 = n1;
    a2 = n2;
}
