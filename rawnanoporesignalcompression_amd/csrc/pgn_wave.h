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

// LDS-only ordering point for a one-wave workgroup.  A wave's DS instructions are executed in order,
// so lanes see each other's earlier LDS writes once the compiler keeps program order: a compiler
// barrier suffices, and nothing waits on the wave's outstanding global loads/stores.
__device__ __forceinline__ void lds_sync()
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// wave prefix sum of 64-bit values
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t x)
{
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    return x;
}

// Global-memory (address space 1) accessors of any alignment.  Every HBM pointer in these kernels
// is global; saying so keeps the compiler from emitting flat instructions, which it must assume may
// alias LDS (and so serialises them against DS traffic and counts them on both vmcnt and lgkmcnt).
template <class T>
struct __attribute__((packed)) Unal {
    T v;
};
#define PGN_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const void* p)
{
    return ((const PGN_GLOBAL Unal<T>*)p)->v;
}
template <class T>
__device__ __forceinline__ void gst(void* p, T v)
{
    ((PGN_GLOBAL Unal<T>*)p)->v = v;
}
__device__ __forceinline__ uint8_t gb(const uint8_t* p) { return *(const PGN_GLOBAL uint8_t*)p; }
// 16-byte forms (HIP's uint4 is not trivially copyable through an address-space-qualified lvalue)
typedef unsigned int pgn_u32x4 __attribute__((ext_vector_type(4)));
template <>
__device__ __forceinline__ uint4 gld<uint4>(const void* p)
{
    const pgn_u32x4 v = ((const PGN_GLOBAL Unal<pgn_u32x4>*)p)->v;
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <>
__device__ __forceinline__ void gst<uint4>(void* p, uint4 v)
{
    pgn_u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    ((PGN_GLOBAL Unal<pgn_u32x4>*)p)->v = t;
}

// unaligned little-endian loads (gfx950 global memory accepts unaligned dword accesses)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) { return gld<uint32_t>(p); }
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) { return gld<uint64_t>(p); }

// byte copy / fill by the whole wave (dst and src may have any alignment; no overlap)
__device__ inline void wave_copy(uint8_t* dst, const uint8_t* src, size_t n)
{
    const int lane = lane_id();
    size_t i = (size_t)lane * 16;
    for (; i + 16 <= n; i += 1024) gst<uint4>(dst + i, gld<uint4>(src + i));
    for (size_t b = (n & ~(size_t)15) + (size_t)lane; b < n; b += 64) gst<uint8_t>(dst + b, gb(src + b));
}
__device__ inline void wave_fill(uint8_t* dst, uint8_t v, size_t n)
{
    for (size_t i = lane_id(); i < n; i += 64) gst<uint8_t>(dst + i, v);
}

// ---------------------------------------------------------------------------------------------
// Optional phase timers (diagnostic builds of a run: PGN_PHASE_PROFILE=1 in the environment).
// Shader-clock cycles accumulate per phase in wave-uniform registers; lane 0 adds them to a global
// buffer at kernel end.  With a null buffer every call is a predictable uniform branch.
// ---------------------------------------------------------------------------------------------
constexpr int kPhases = 16;
struct PhaseProf {
    uint64_t* out;
    uint64_t last;
    uint64_t acc[kPhases];
    __device__ void init(uint64_t* o)
    {
        out = o;
        for (int i = 0; i < kPhases; i++) acc[i] = 0;
        last = o ? __builtin_amdgcn_s_memtime() : 0;
    }
    __device__ __forceinline__ void mark(int phase)
    {
        if (out) {
            uint64_t t = __builtin_amdgcn_s_memtime();
            acc[phase] += t - last;
            last = t;
        }
    }
    __device__ void flush()
    {
        if (out && lane_id() == 0)
            for (int i = 0; i < kPhases; i++) atomicAdd((unsigned long long*)&out[i], (unsigned long long)acc[i]);
    }
};

}  // namespace pgn
