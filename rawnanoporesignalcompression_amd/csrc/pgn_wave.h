// pgn_wave.h -- wave64 building blocks for the gfx950 kernels (one 64-lane wavefront owns one
// POD5 signal chunk; see DESIGN.md "Kernels").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pgn {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l)
{
    uint32_t lo = readlane_u32((uint32_t)v, l), hi = readlane_u32((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// inclusive / exclusive prefix sums across the wave
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x)
{
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) { return readlane_u32(wave_incl_sum(x), 63); }
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t t = __shfl_xor(x, d, 64);
        x = t > x ? t : x;
    }
    return x;
}

// one-wave workgroup barrier that also orders global/LDS memory for the wave's lanes
__device__ __forceinline__ void wave_sync() { __syncthreads(); }

// unaligned little-endian loads (gfx950 global memory accepts unaligned dword accesses)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p)
{
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p)
{
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// byte copy / fill by the whole wave (dst and src may have any alignment; no overlap)
__device__ inline void wave_copy(uint8_t* dst, const uint8_t* src, size_t n)
{
    const int lane = lane_id();
    size_t i = (size_t)lane * 4;
    for (; i + 4 <= n; i += 256) {
        uint32_t v = ld32u(src + i);
        __builtin_memcpy(dst + i, &v, 4);
    }
    size_t tail = n & ~(size_t)3;
    if ((size_t)lane < n - tail) dst[tail + lane] = src[tail + lane];
}
__device__ inline void wave_fill(uint8_t* dst, uint8_t v, size_t n)
{
    for (size_t i = lane_id(); i < n; i += 64) dst[i] = v;
}

}  // namespace pgn
