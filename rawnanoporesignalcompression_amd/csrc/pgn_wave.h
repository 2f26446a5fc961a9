// pgn_wave.h -- wave64 building blocks for the gfx950 kernels (one 64-lane wavefront owns one
// POD5 signal chunk; see DESIGN.md "Kernels").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pgn {

// The encoder's and the decoder's wave workspaces (EncLds in pgn_zenc.h, DecLds in pgn_zdec.h) are
// one LDS variable.  Two variables named by non-kernel functions of different kernel sets make LLVM's
// LDS lowering keep only one of them at a fixed address and reach the other through a per-kernel
// offset table (a scalar load on its access paths; which one depends on how many kernels reach
// each, so adding a decode kernel moved the encoder's behind the table: encode +4 %).  One variable
// reached by every codec kernel sits at offset 0 in each of them.
constexpr size_t kCodecLdsBytes = 8192;
// an LDS word pointer (cooperative kernels pass their own LDS to the shared device functions this way)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
static __shared__ __attribute__((aligned(16))) uint8_t sCodecLds[kCodecLdsBytes];

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

// Wave-uniform values.  Arguments of a non-inlined device function arrive in VGPRs and are treated
// as divergent; passing the wave-uniform ones through readfirstlane at entry gives the compiler
// scalar registers, scalar loop control and scalar address arithmetic back.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni(uint64_t v)
{
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
__device__ __forceinline__ long uni(long v) { return (long)uni((uint64_t)v); }
template <class T>
__device__ __forceinline__ T* uni(T* p)
{
    return (T*)uni((uint64_t)p);
}

// DPP lane moves (GFX9 encodings; gfx950 keeps the row_bcast / wave_shr controls of GFX9).
// Lanes without a source read 0.
enum : int {
    kDppQuadSwap1 = 0xB1,   // quad_perm [1,0,3,2]
    kDppQuadSwap2 = 0x4E,   // quad_perm [2,3,0,1]
    kDppRowShr1 = 0x111,
    kDppRowShr2 = 0x112,
    kDppRowShr4 = 0x114,
    kDppRowShr8 = 0x118,
    kDppWaveShr1 = 0x138,
    kDppRowBcast15 = 0x142,
    kDppRowBcast31 = 0x143,
};
template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, 0xF, true);
}

// number of set bits of m below this lane
__device__ __forceinline__ uint32_t mbcnt(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// inclusive prefix sum across the wave (DPP: 4 in-row steps + 2 row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x)
{
    x += dpp<kDppRowShr1>(x);
    x += dpp<kDppRowShr2>(x);
    x += dpp<kDppRowShr4>(x);
    x += dpp<kDppRowShr8>(x);
    x += dpp<kDppRowBcast15, 0xA>(x);
    x += dpp<kDppRowBcast31, 0xC>(x);
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

// Ordering point between the lanes of a one-wave workgroup.  The lanes of a wavefront are coherent
// through LDS and the CU's vector L1 without waits (a wave's DS and vector-memory instructions are
// performed in program order; LLVM AMDGPU memory model, gfx942/gfx950), so keeping program order in
// the compiler suffices.  In particular no s_waitcnt vmcnt(0): a __syncthreads() here would stall
// every call site until the wave's outstanding HBM stores drain.
__device__ __forceinline__ void lds_sync()
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void wave_sync() { lds_sync(); }

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

// Non-temporal 16-byte store (the nt bit: data written once is not kept in the caches at the expense
// of data that is reused); 16-byte aligned addresses only.
__device__ __forceinline__ void gst_nt16(void* p, uint4 v)
{
    pgn_u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    __builtin_nontemporal_store(t, (PGN_GLOBAL pgn_u32x4*)p);
}

// wave_copy with non-temporal stores (the destination is not read again soon); any alignment: the
// head bytes up to dst's first 16-byte boundary one per lane, then aligned 16-byte stores
__device__ inline void wave_copy_nt(uint8_t* dst, const uint8_t* src, size_t n)
{
    const int lane = lane_id();
    const size_t head = ((16u - ((uintptr_t)dst & 15u)) & 15u) < n ? ((16u - ((uintptr_t)dst & 15u)) & 15u) : n;
    if ((size_t)lane < head) gst<uint8_t>(dst + lane, gb(src + lane));
    dst += head;
    src += head;
    n -= head;
    size_t i = (size_t)lane * 16;
    for (; i + 16 + 3 * 1024 <= n; i += 4096) {
        const uint4 a = gld<uint4>(src + i), b = gld<uint4>(src + i + 1024), c = gld<uint4>(src + i + 2048),
                    d = gld<uint4>(src + i + 3072);
        gst_nt16(dst + i, a);
        gst_nt16(dst + i + 1024, b);
        gst_nt16(dst + i + 2048, c);
        gst_nt16(dst + i + 3072, d);
    }
    for (; i + 16 <= n; i += 1024) gst_nt16(dst + i, gld<uint4>(src + i));
    for (size_t k = (n & ~(size_t)15) + (size_t)lane; k < n; k += 64) gst<uint8_t>(dst + k, gb(src + k));
}

// unaligned little-endian loads (gfx950 global memory accepts unaligned dword accesses)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) { return gld<uint32_t>(p); }
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) { return gld<uint64_t>(p); }

// byte copy / fill by the whole wave (dst and src may have any alignment; no overlap)
__device__ inline void wave_copy(uint8_t* dst, const uint8_t* src, size_t n)
{
    const int lane = lane_id();
    size_t i = (size_t)lane * 16;
    for (; i + 16 + 3 * 1024 <= n; i += 4096) {  // four 16-byte loads in flight per lane
        const uint4 a = gld<uint4>(src + i), b = gld<uint4>(src + i + 1024), c = gld<uint4>(src + i + 2048),
                    d = gld<uint4>(src + i + 3072);
        gst<uint4>(dst + i, a);
        gst<uint4>(dst + i + 1024, b);
        gst<uint4>(dst + i + 2048, c);
        gst<uint4>(dst + i + 3072, d);
    }
    for (; i + 16 <= n; i += 1024) gst<uint4>(dst + i, gld<uint4>(src + i));
    for (size_t b = (n & ~(size_t)15) + (size_t)lane; b < n; b += 64) gst<uint8_t>(dst + b, gb(src + b));
}
// the same with eight 16-byte loads in flight per lane (8 KiB per wave round trip): large copies
// such as a raw block are latency-bound on the number of round trips
__device__ inline void wave_copy8(uint8_t* dst, const uint8_t* src, size_t n)
{
    const size_t l16 = (size_t)lane_id() * 16;
    size_t base = 0;  // wave-uniform: whole 8 KiB rounds, then wave_copy for the rest
    for (; base + 8192 <= n; base += 8192) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = gld<uint4>(src + base + l16 + 1024 * k);
#pragma unroll
        for (int k = 0; k < 8; k++) gst<uint4>(dst + base + l16 + 1024 * k, v[k]);
    }
    wave_copy(dst + base, src + base, n - base);
}
__device__ inline void wave_fill(uint8_t* dst, uint8_t v, size_t n)
{
    for (size_t i = lane_id(); i < n; i += 64) gst<uint8_t>(dst + i, v);
}

// ---------------------------------------------------------------------------------------------
// Optional phase timers, compiled only into the diagnostic build of the library (PGN_PROFILE;
// `_build/libpgnano_hip_prof.so`, selected with PGN_PHASE_PROFILE=1).  Shader-clock cycles
// accumulate per phase; lane 0 adds them to a global buffer at kernel end.
// ---------------------------------------------------------------------------------------------
constexpr int kPhases = 16;
constexpr int kCounters = 16;  // event counters (loop trip counts) after the phase cycles
// profile buffer: [encode phases][decode phases][encode counters][decode counters], then the same
// pair for dec_huf_kernel (phases at kHufProfOff, counters 2 kPhases further on)
constexpr int kHufProfOff = 2 * (kPhases + kCounters);
constexpr int kProfWords = kHufProfOff + 2 * (kPhases + kCounters);
struct PhaseProf {
#ifdef PGN_PROFILE
    uint64_t* out;
    uint64_t last;
    uint64_t acc[kPhases];
    uint64_t cnt[kCounters];
    __device__ void init(uint64_t* o)
    {
        out = o;
        for (int i = 0; i < kPhases; i++) acc[i] = 0;
        for (int i = 0; i < kCounters; i++) cnt[i] = 0;
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
    // wave-level event count (call with wave-uniform control flow)
    __device__ __forceinline__ void count(int k, uint64_t v = 1)
    {
        if (out) cnt[k] += v;
    }
    __device__ void flush()
    {
        if (out && lane_id() == 0) {
            for (int i = 0; i < kPhases; i++) atomicAdd((unsigned long long*)&out[i], (unsigned long long)acc[i]);
            for (int i = 0; i < kCounters; i++)
                atomicAdd((unsigned long long*)&out[2 * kPhases + i], (unsigned long long)cnt[i]);
        }
    }
#else
    __device__ __forceinline__ void init(uint64_t*) {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void count(int, uint64_t = 1) {}
    __device__ __forceinline__ void flush() {}
#endif
};

}  // namespace pgn
