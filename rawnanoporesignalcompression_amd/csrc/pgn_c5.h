// pgn_c5.h -- C5 ("N01") split and merge on one wave.
//
// Split = svb16::encode_scalar_N01<int16_t, /*delta*/true, /*zigzag*/true> (pgnano/svb16/C5.hpp:57-152)
// Merge = svb16::decode_scalar_N01 (C5.hpp:173-257) as driven by decode_N01 (C5.hpp:260-275) and
//         decompress_signal_N01's consumed-bytes check (C5.hpp:669-677).
//
// The reference walks the samples serially; here a wave takes 1024 samples per step, one sample per
// lane per sub-step: class ballots and mbcnt ranks place every S/M/L byte, LDS windows turn the
// scattered bytes into aligned 16-byte HBM stores, and a DPP wave scan undoes the 16-bit delta.
#pragma once
#include "pgn_wave.h"

namespace pgn {

__device__ __forceinline__ uint16_t zz_enc16(uint16_t v) { return (uint16_t)((uint16_t)(v + v) ^ (uint16_t)((int16_t)v >> 15)); }
__device__ __forceinline__ uint16_t zz_dec16(uint16_t v) { return (uint16_t)((v >> 1) ^ (uint16_t)(0u - (v & 1u))); }

struct C5Streams {
    uint8_t *K, *S, *M, *Ll, *Lh;
};

// ---------------------------------------------------------------------------------------------
// Split.  A step is 1024 samples; lane l takes the 16 consecutive samples t + 16l .. t + 16l + 15,
// so its 16 keys are one key word.  A value's place in its stream is the stream's fill plus the
// class counts of the lanes below (one packed DPP scan) plus its rank among the lane's own
// samples, so each lane writes its bytes straight into LDS windows (bytes of other classes go to
// a per-lane dummy slot instead of being predicated).  After a step, complete 16-byte blocks of
// each window go to HBM as aligned 16-byte stores and the tail moves to the window front.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kSplitStep = 1024;
constexpr uint32_t kWinBytes = 1088;  // 31 carried nibbles + 1024 new, rounded up to 16

struct SplitLds {
    alignas(16) uint8_t S[kWinBytes + 256];  // one byte per nibble
    alignas(16) uint8_t M[kWinBytes + 256];
    alignas(16) uint8_t L[kWinBytes];
    alignas(16) uint8_t H[kWinBytes];
    alignas(16) uint32_t Z[64 * 8];  // a lane's 16 zig-zag values (two per word), for its class-3 samples
    alignas(16) uint8_t D[64 * 16];  // a lane's 16 discard bytes (what its class-0 / class-3 samples write)
};

typedef uint16_t pgn_u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t pgn_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pgn_u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(pgn_u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(pgn_u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// packed 16-bit min / saturating subtract / wrapping subtract (one VOP3P instruction each)
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "s"(b));
    return r;
}
__device__ __forceinline__ uint32_t pk_subsat_u16(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "s"(b));
    return r;
}
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// 4 nibble-bytes (each < 16) -> their 16-bit little-endian nibble packing
__device__ __forceinline__ uint32_t pack_nibbles(uint32_t w)
{
    const uint32_t y = w | (w >> 4);
    return (y & 0xFFu) | ((y >> 8) & 0xFF00u);
}

// flush the complete 16-byte blocks of a byte window to out + gpos (gpos % 16 == 0)
__device__ __forceinline__ void bwin_flush(uint8_t* W, uint32_t& fill, uint8_t* out, uint32_t& gpos)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t nblk = fill >> 4, tail = fill & 15u;
    for (uint32_t b = lane; b < nblk; b += 64) gst<uint4>(out + gpos + 16u * b, *(const uint4*)(W + 16u * b));
    if (nblk) {
        const uint8_t v = W[16u * nblk + (lane & 15u)];
        if (lane < tail) W[lane] = v;
    }
    gpos += 16u * nblk;
    fill = tail;
}

// the same for the nibble window: 32 nibble-bytes make 16 output bytes
__device__ __forceinline__ void nwin_flush(uint8_t* W, uint32_t& fill, uint8_t* out, uint32_t& gpos)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t nblk = fill >> 5, tail = fill & 31u;
    for (uint32_t b = lane; b < nblk; b += 64) {
        const uint4 a = *(const uint4*)(W + 32u * b), c = *(const uint4*)(W + 32u * b + 16u);
        uint4 o;
        o.x = pack_nibbles(a.x) | (pack_nibbles(a.y) << 16);
        o.y = pack_nibbles(a.z) | (pack_nibbles(a.w) << 16);
        o.z = pack_nibbles(c.x) | (pack_nibbles(c.y) << 16);
        o.w = pack_nibbles(c.z) | (pack_nibbles(c.w) << 16);
        gst<uint4>(out + gpos + 16u * b, o);
    }
    if (nblk) {
        const uint8_t v = W[32u * nblk + (lane & 31u)];
        if (lane < tail) W[lane] = v;
    }
    gpos += 16u * nblk;
    fill = tail;
}

// Class offsets: C5 (N01) stores v-1 / v-17 / v-273 (C5.hpp:105-140); C4 (N02, C4.hpp:100-133)
// stores the raw value, classes v < 16 / v < 256 / else.
template <bool C4> struct ClassOffsets {
    static constexpr uint32_t o1 = C4 ? 0u : 1u, o2 = C4 ? 0u : 17u, o3 = C4 ? 0u : 273u;
    static constexpr uint32_t t1 = C4 ? 15u : 16u, t2 = C4 ? 255u : 272u;  // class >= 2 iff v > t1, 3 iff v > t2
};

// (m & a) | (~m & b) as one v_bfi_b32 (written as and/or or ?:, the selects become compare +
// cndmask pairs)
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// One 1024-sample step (Full: every sample of the step exists).  Returns the lane's key word.
// Full steps take the lane's 32 sample bytes already loaded (a, b: prefetched one step ahead).
// Deltas, zig-zag and classes are computed two samples per instruction (packed 16-bit halves):
// class = (v >= 1) + (v > t1) + (v > t2) from saturating subtracts.
template <bool Full, bool C4 = false>
__device__ __forceinline__ uint32_t split_step(const uint4& a, const uint4& b, const int16_t* __restrict__ x, uint32_t n,
                                               uint32_t t, SplitLds& W, uint32_t& fS, uint32_t& fM, uint32_t& fL,
                                               uint32_t& prevX)
{
    using CO = ClassOffsets<C4>;
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t i0 = t + 16u * lane;
    uint32_t wd[8];
    if (Full) {
        wd[0] = a.x; wd[1] = a.y; wd[2] = a.z; wd[3] = a.w;
        wd[4] = b.x; wd[5] = b.y; wd[6] = b.z; wd[7] = b.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t lo = (i0 + 2u * k < n) ? (uint32_t)gld<uint16_t>(x + i0 + 2 * k) : 0u;
            const uint32_t hi = (i0 + 2u * k + 1u < n) ? (uint32_t)gld<uint16_t>(x + i0 + 2 * k + 1) : 0u;
            wd[k] = lo | (hi << 16);
        }
    }
    // the sample before mine: lane l-1's last one (lane 0: the previous step's)
    uint32_t prv = dpp<kDppWaveShr1>(wd[7] >> 16);
    prv = (lane == 0) ? prevX : prv;
    prevX = readlane_u32(wd[7] >> 16, 63);
    constexpr uint32_t kOne = 0x00010001u, kT1 = CO::t1 * kOne, kT2 = CO::t2 * kOne;
    // stage by stage over the 8 pairs, so that dependent packed instructions are never adjacent
    uint32_t z[8], val[8], cp[8], c2[8], c3[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t before = (k == 0) ? ((wd[0] << 16) | prv) : __builtin_amdgcn_alignbit(wd[k], wd[k - 1], 16);
        const pgn_u16x2 d = as_u16x2(wd[k]) - as_u16x2(before);
        z[k] = as_u32((d << (pgn_u16x2){1, 1}) ^ __builtin_bit_cast(pgn_u16x2, __builtin_bit_cast(pgn_s16x2, d) >> (pgn_s16x2){15, 15}));
    }
#pragma unroll
    for (int k = 0; k < 8; k++) c2[k] = pk_subsat_u16(z[k], kT1);
#pragma unroll
    for (int k = 0; k < 8; k++) c3[k] = pk_subsat_u16(z[k], kT2);
#pragma unroll
    for (int k = 0; k < 8; k++) cp[k] = pk_min_u16(z[k], kOne);
#pragma unroll
    for (int k = 0; k < 8; k++) c2[k] = pk_min_u16(c2[k], kOne);
#pragma unroll
    for (int k = 0; k < 8; k++) c3[k] = pk_min_u16(c3[k], kOne);
#pragma unroll
    for (int k = 0; k < 8; k++) {
        cp[k] += c2[k] + c3[k];  // halves <= 3: no carry between them
        if (!Full) {
            const uint32_t vm = ((i0 + 2u * k < n) ? 0xFFFFu : 0u) | ((i0 + 2u * k + 1u < n) ? 0xFFFF0000u : 0u);
            cp[k] &= vm;
        }
    }
    // the byte a class-1 / class-2 sample stores: v - o1 or v - o2
#pragma unroll
    for (int k = 0; k < 8; k++) val[k] = C4 ? z[k] : pk_sub_u16(z[k], kOne + (c2[k] << 4));
    // key word: sample m's class at bits 2m (pairs k: low half -> 4k, high half -> 4k + 2)
    const uint32_t X = cp[0] | (cp[1] << 4) | (cp[2] << 8) | (cp[3] << 12);
    const uint32_t Y = cp[4] | (cp[5] << 4) | (cp[6] << 8) | (cp[7] << 12);
    const uint32_t Xn = (X & 0x3333u) | ((X >> 14) & 0xCCCCu), Yn = (Y & 0x3333u) | ((Y >> 14) & 0xCCCCu);
    const uint32_t kw = Xn | (Yn << 16);
    // places: step fills + the classes of the lanes below (one packed scan) + ranks within the lane
    const uint32_t lo = kw & 0x55555555u, hi = (kw >> 1) & 0x55555555u;
    const uint32_t m1 = lo & ~hi, m2 = hi & ~lo, m3 = lo & hi;
    const uint32_t pc = (uint32_t)__builtin_popcount(m1) | ((uint32_t)__builtin_popcount(m2) << 11) |
                        ((uint32_t)__builtin_popcount(m3) << 22);
    const uint32_t inc = wave_incl_sum(pc);
    const uint32_t tot = readlane_u32(inc, 63);
    const uint32_t exc = inc - pc;
    uint8_t* const wb = reinterpret_cast<uint8_t*>(&W);
    constexpr uint32_t offS = (uint32_t)__builtin_offsetof(SplitLds, S), offM = (uint32_t)__builtin_offsetof(SplitLds, M);
    const uint32_t baseS = offS + fS + (exc & 0x7FFu), baseM = offM + fM + ((exc >> 11) & 0x7FFu);
    // the lane's four next places as the 16-bit fields of one 64-bit word, field c = class c (classes
    // 0 and 3 write the lane's discard bytes): sample m's place is field c_m (one v_perm_b32), and
    // that field advances by one byte (1 << 16 c_m)
    constexpr uint32_t offD = (uint32_t)__builtin_offsetof(SplitLds, D);
    static_assert(sizeof(SplitLds) < 65536, "split places are 16-bit");
    const uint32_t dD = offD + 16u * lane;
    uint32_t plo = dD | (baseS << 16), phi = baseM | (dD << 16);
#pragma unroll
    for (int m = 0; m < 16; m++) {
        const uint32_t c = __builtin_amdgcn_ubfe(kw, 2 * m, 2);
        const uint32_t at = __builtin_amdgcn_perm(phi, plo, c * 0x0202u + 0x0C0C0100u);
        if (m < 15) {
            const uint64_t inc = (uint64_t)1 << (16 * c);
            plo += (uint32_t)inc;
            phi += (uint32_t)(inc >> 32);
        }
        wb[at] = (uint8_t)(val[m >> 1] >> (16 * (m & 1)));
    }
    // field 3 has 10 bits: a step of 1024 class-3 samples wraps the inclusive total (the exclusive
    // prefixes stay exact), so its total is rebuilt from the last lane
    const uint32_t t3 = (readlane_u32(exc, 63) >> 22) + (readlane_u32(pc, 63) >> 22);
    if (t3) {  // class 3 is rare: each lane walks its own class-3 samples, values from an LDS stash
        if (m3) {
#pragma unroll
            for (int k = 0; k < 8; k++) W.Z[8 * lane + k] = z[k];
            uint32_t qL = fL + (exc >> 22);
            const uint16_t* zs = reinterpret_cast<const uint16_t*>(W.Z) + 16 * lane;
            for (uint32_t mm = m3; mm; mm &= mm - 1u) {
                const uint32_t w = (uint32_t)zs[__builtin_ctz(mm) >> 1] - CO::o3;
                W.L[qL] = (uint8_t)w;
                W.H[qL] = (uint8_t)(w >> 8);
                qL++;
            }
        }
    }
    fS += tot & 0x7FFu;
    fM += (tot >> 11) & 0x7FFu;
    fL += t3;
    return kw;
}

// sizes[5] = {keys, S, M, Llow, Lhigh} bytes.  C4: the N02 variant (same layout, raw values).
template <bool C4 = false>
__device__ __forceinline__ void c5_split_wave(const int16_t* __restrict__ x, uint32_t n, const C5Streams& st, uint32_t sizes[5],
                                              SplitLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t fS = 0, fM = 0, fL = 0, fH = 0;  // window fills (S in nibbles)
    uint32_t gS = 0, gM = 0, gL = 0, gH = 0;  // bytes already in HBM
    uint32_t prevX = 0;                       // last sample of the previous sub-step (wave-uniform)
    // the samples of a full step are loaded one step ahead, so their latency overlaps a step
    uint4 na = make_uint4(0u, 0u, 0u, 0u), nb = na;
    auto ld16 = [&](const int16_t* p) { return gld<uint4>(p); };
    if (kSplitStep <= n) {
        na = ld16(x + 16u * lane);
        nb = ld16(x + 16u * lane + 8);
    }
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        const uint4 ca = na, cb = nb;
        if (t + 2 * kSplitStep <= n) {
            na = ld16(x + t + kSplitStep + 16u * lane);
            nb = ld16(x + t + kSplitStep + 16u * lane + 8);
        }
        const uint32_t kw = full ? split_step<true, C4>(ca, cb, x, n, t, W, fS, fM, fL, prevX)
                                 : split_step<false, C4>(ca, cb, x, n, t, W, fS, fM, fL, prevX);
        fH = fL;
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        uint8_t* kout = st.K + (t >> 2);
        if (4u * lane + 4u <= nK) gst<uint32_t>(kout + 4u * lane, kw);
        else for (uint32_t b = 4u * lane; b < nK; b++) gst<uint8_t>(kout + b, (uint8_t)(kw >> (8u * (b - 4u * lane))));
        lds_sync();
        nwin_flush(W.S, fS, st.S, gS);
        bwin_flush(W.M, fM, st.M, gM);
        bwin_flush(W.L, fL, st.Ll, gL);
        bwin_flush(W.H, fH, st.Lh, gH);
        lds_sync();
    }
    // tails (a trailing odd nibble leaves its high half zero)
    const uint32_t nbS = (fS + 1) / 2;
    for (uint32_t j = lane; j < nbS; j += 64) {
        const uint32_t lo = W.S[2 * j], hi = (2 * j + 1 < fS) ? W.S[2 * j + 1] : 0u;
        gst<uint8_t>(st.S + gS + j, (uint8_t)(lo | (hi << 4)));
    }
    for (uint32_t j = lane; j < fM; j += 64) gst<uint8_t>(st.M + gM + j, W.M[j]);
    for (uint32_t j = lane; j < fL; j += 64) {
        gst<uint8_t>(st.Ll + gL + j, W.L[j]);
        gst<uint8_t>(st.Lh + gH + j, W.H[j]);
    }
    lds_sync();
    sizes[0] = (n + 3) / 4;
    sizes[1] = gS + nbS;
    sizes[2] = gM + fM;
    sizes[3] = gL + fL;
    sizes[4] = gL + fL;
}

// ---------------------------------------------------------------------------------------------
// Split of a step range [t0, t1) (small batches: the waves of a workgroup share one chunk).  The
// range's streams start at S nibble pS and M / class-3 bytes pM / pL (the class counts of the
// ranges before it); its windows start at the 16-byte block holding that first entry, and the
// entries in front of it ("lead", the ranges before) are never written.  The S byte shared with the
// range before (pS odd) and a trailing half byte are left to the caller, with the nibbles it needs:
// firstNib (the range's first nibble when pS is odd) and lastNib (its last when its end is odd);
// 0xFF for none.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void bwin_flush_lead(uint8_t* W, uint32_t& fill, uint8_t* out, uint32_t& gpos, uint32_t& lead)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t nblk = fill >> 4, tail = fill & 15u;
    for (uint32_t b = lane; b < nblk; b += 64) {
        if (b == 0 && lead) {
            for (uint32_t k = lead; k < 16; k++) gst<uint8_t>(out + gpos + k, W[k]);
        } else {
            gst<uint4>(out + gpos + 16u * b, *(const uint4*)(W + 16u * b));
        }
    }
    if (nblk) {
        const uint8_t v = W[16u * nblk + (lane & 15u)];
        if (lane < tail) W[lane] = v;
        lead = 0;
    }
    gpos += 16u * nblk;
    fill = tail;
}
__device__ __forceinline__ void nwin_flush_lead(uint8_t* W, uint32_t& fill, uint8_t* out, uint32_t& gpos, uint32_t& lead)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t nblk = fill >> 5, tail = fill & 31u;
    for (uint32_t b = lane; b < nblk; b += 64) {
        if (b == 0 && lead) {  // bytes whose both nibbles are the range's (the shared one is the caller's)
            for (uint32_t k = (lead + 1) >> 1; k < 16; k++) gst<uint8_t>(out + gpos + k, (uint8_t)(W[2 * k] | (W[2 * k + 1] << 4)));
        } else {
            const uint4 a = *(const uint4*)(W + 32u * b), c = *(const uint4*)(W + 32u * b + 16u);
            uint4 o;
            o.x = pack_nibbles(a.x) | (pack_nibbles(a.y) << 16);
            o.y = pack_nibbles(a.z) | (pack_nibbles(a.w) << 16);
            o.z = pack_nibbles(c.x) | (pack_nibbles(c.y) << 16);
            o.w = pack_nibbles(c.z) | (pack_nibbles(c.w) << 16);
            gst<uint4>(out + gpos + 16u * b, o);
        }
    }
    if (nblk) {
        const uint8_t v = W[32u * nblk + (lane & 31u)];
        if (lane < tail) W[lane] = v;
        lead = 0;
    }
    gpos += 16u * nblk;
    fill = tail;
}

template <bool C4 = false>
__device__ inline void c5_split_range(const int16_t* __restrict__ x, uint32_t n, uint32_t t0, uint32_t t1,
                                      const C5Streams& st, uint32_t pS, uint32_t pM, uint32_t pL, SplitLds& W,
                                      uint32_t& firstNib, uint32_t& lastNib)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t fS = pS & 31u, fM = pM & 15u, fL = pL & 15u, fH = fL;  // window fills, lead included
    uint32_t gS = (pS >> 1) & ~15u, gM = pM & ~15u, gL = pL & ~15u, gH = gL;
    uint32_t leadS = fS, leadM = fM, leadL = fL, leadH = fL;
    uint32_t prevX = t0 ? (uint32_t)(uint16_t)__builtin_amdgcn_readfirstlane((int)gld<uint16_t>(x + t0 - 1)) : 0u;
    firstNib = 0xFFu;
    lastNib = 0xFFu;
    uint4 na = make_uint4(0u, 0u, 0u, 0u), nb = na;
    if (t0 + kSplitStep <= n) {
        na = gld<uint4>(x + t0 + 16u * lane);
        nb = gld<uint4>(x + t0 + 16u * lane + 8);
    }
    for (uint32_t t = t0; t < t1; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        const uint4 ca = na, cb = nb;
        if (t + kSplitStep < t1 && t + 2 * kSplitStep <= n) {
            na = gld<uint4>(x + t + kSplitStep + 16u * lane);
            nb = gld<uint4>(x + t + kSplitStep + 16u * lane + 8);
        }
        const uint32_t kw = full ? split_step<true, C4>(ca, cb, x, n, t, W, fS, fM, fL, prevX)
                                 : split_step<false, C4>(ca, cb, x, n, t, W, fS, fM, fL, prevX);
        fH = fL;
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        uint8_t* kout = st.K + (t >> 2);
        if (4u * lane + 4u <= nK) gst<uint32_t>(kout + 4u * lane, kw);
        else for (uint32_t b = 4u * lane; b < nK; b++) gst<uint8_t>(kout + b, (uint8_t)(kw >> (8u * (b - 4u * lane))));
        lds_sync();
        if (firstNib == 0xFFu && (pS & 1u) && fS > leadS) firstNib = W.S[leadS];
        nwin_flush_lead(W.S, fS, st.S, gS, leadS);
        bwin_flush_lead(W.M, fM, st.M, gM, leadM);
        bwin_flush_lead(W.L, fL, st.Ll, gL, leadL);
        bwin_flush_lead(W.H, fH, st.Lh, gH, leadH);
        lds_sync();
    }
    // tails: whole bytes of the range only
    const uint32_t nbS = (fS + 1) / 2;
    for (uint32_t j = lane; j < nbS; j += 64) {
        if (2 * j < leadS || 2 * j + 1 >= fS) continue;  // the lead's, the shared byte, or a trailing half byte
        gst<uint8_t>(st.S + gS + j, (uint8_t)(W.S[2 * j] | (W.S[2 * j + 1] << 4)));
    }
    if (fS > leadS && (fS & 1u)) lastNib = W.S[fS - 1];
    for (uint32_t j = leadM + lane; j < fM; j += 64) gst<uint8_t>(st.M + gM + j, W.M[j]);
    for (uint32_t j = leadL + lane; j < fL; j += 64) {
        gst<uint8_t>(st.Ll + gL + j, W.L[j]);
        gst<uint8_t>(st.Lh + gH + j, W.H[j]);
    }
    lds_sync();
}

// Class counts (S, M, class 3) of the samples [t0, t1) of a chunk, from the samples (the delta of
// sample 0 is from 0), wave-uniform.
template <bool C4 = false>
__device__ inline void c5_split_counts(const int16_t* __restrict__ x, uint32_t n, uint32_t t0, uint32_t t1, uint32_t& cS,
                                       uint32_t& cM, uint32_t& cL)
{
    using CO = ClassOffsets<C4>;
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t s = 0, m = 0, l = 0;
    // four 1,024-sample steps per trip, their loads issued together (the pass is latency-bound)
    for (uint32_t tb = t0; tb < t1; tb += 4096u) {
        uint32_t wv[4][8], pv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + 1024u * u + 16u * lane;
            pv[u] = (t < t1 && t) ? (uint32_t)gld<uint16_t>(x + t - 1) : 0u;
            if (t + 16u <= t1) {
                const uint4 a = gld<uint4>(x + t), b = gld<uint4>(x + t + 8);
                wv[u][0] = a.x; wv[u][1] = a.y; wv[u][2] = a.z; wv[u][3] = a.w;
                wv[u][4] = b.x; wv[u][5] = b.y; wv[u][6] = b.z; wv[u][7] = b.w;
            } else {
#pragma unroll
                for (uint32_t k = 0; k < 8; k++) {
                    const uint32_t lo = t + 2 * k < t1 ? (uint32_t)gld<uint16_t>(x + t + 2 * k) : 0u;
                    const uint32_t hi = t + 2 * k + 1 < t1 ? (uint32_t)gld<uint16_t>(x + t + 2 * k + 1) : 0u;
                    wv[u][k] = lo | (hi << 16);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + 1024u * u + 16u * lane;
            uint32_t prev = pv[u];
#pragma unroll
            for (uint32_t k = 0; k < 16; k++) {
                const bool in = t + k < t1;
                const uint32_t v = (wv[u][k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                const uint32_t d = (v - prev) & 0xFFFFu;
                const uint32_t z = ((d << 1) ^ (0u - (d >> 15))) & 0xFFFFu;
                prev = v;
                s += (in && z >= 1u && z <= CO::t1) ? 1u : 0u;
                m += (in && z > CO::t1 && z <= CO::t2) ? 1u : 0u;
                l += (in && z > CO::t2) ? 1u : 0u;
            }
        }
    }
    cS = wave_sum(s);
    cM = wave_sum(m);
    cL = wave_sum(l);
}

// ---------------------------------------------------------------------------------------------
// Merge over the reference's concatenated intermediate buffer (see oracle c5_merge): stream starts at
// keys_length = ceil(n/4), then +dS, +dM, +dLl; a read past `total` is the reference's UB -> error.
// Per 1024-sample step the class counts come from the key bytes, the step's S/M/L bytes are staged
// into LDS with 16-byte loads, and each lane decodes 16 consecutive samples (merge_step).  `in`
// must stay readable 16 bytes past `total` (scratch padding).
// Returns 0 ok, 1 out-of-bounds; *consumed = one past the last Lhigh byte.
// ---------------------------------------------------------------------------------------------
struct MergeLds {
    // one step's S, M and class-3 values as 16-bit deltas (class offsets added, zig-zag decoded), back
    // to back: S (one nibble per entry) from a 16-byte aligned stream byte, then M likewise, then L | H << 8.
    // A step has at most 1024 of them together, plus the alignment slack of two windows.
    alignas(16) uint16_t V[1024 + 64 + 32 + 32];
    uint16_t zero[16];  // what class-0 samples read (a lane's place here advances with them)
    // S byte -> its two entries (low nibble first), offset added and zig-zag decoded
    alignas(16) uint32_t nib[256];
};

static_assert(sizeof(MergeLds) < 65536, "merge places are 16-bit");

// stage bytes [a, a + len) of `in` (len <= cap - 15) into W; returns the window's first address
__device__ __forceinline__ uint64_t stage_bytes(uint8_t* W, const uint8_t* in, uint64_t a, uint32_t len)
{
    const uint64_t a0 = a & ~(uint64_t)15;
    const uint32_t nblk = (uint32_t)((a + len - a0 + 15) >> 4);
    for (uint32_t b = (uint32_t)lane_id(); b < nblk; b += 64) *(uint4*)(W + 16u * b) = gld<uint4>(in + a0 + 16u * b);
    return a0;
}

// two zig-zag codes -> their 16-bit deltas (packed)
__device__ __forceinline__ uint32_t zz_dec16x2(uint32_t w)
{
    const pgn_u16x2 x = as_u16x2(w);
    return as_u32((x >> (pgn_u16x2){1, 1}) ^ ((pgn_u16x2){0, 0} - (x & (pgn_u16x2){1, 1})));
}
// 16 bytes -> 16 entries + add, zig-zag decoded, written at d
__device__ __forceinline__ void put_bytes16(uint16_t* d, const uint4& v, uint32_t add2)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        o[2 * j] = zz_dec16x2(__builtin_amdgcn_perm(0u, w[j], 0x0C010C00u) + add2);
        o[2 * j + 1] = zz_dec16x2(__builtin_amdgcn_perm(0u, w[j], 0x0C030C02u) + add2);
    }
    uint4* q = (uint4*)d;
    q[0] = make_uint4(o[0], o[1], o[2], o[3]);
    q[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// Merge step over 1024 samples: lane l decodes the 16 consecutive samples t + 16l .. t + 16l + 15,
// whose 16 keys are its own key word.  Every class has a staged 16-bit window of deltas (offsets
// added and zig-zag decoded at staging; class 0 reads zeros), and the lane's first place in each is
// the step's fill plus the class counts of the lanes below it (one packed DPP scan).  The lane keeps
// its four next places as the 16-bit fields of one 64-bit word, field c = class c: sample m's place
// is field c_m (one v_perm_b32 whose selector is c_m * 0x0202 + 0x0C0C0100), and the field advances
// by one entry (2 << 16 c_m, a 64-bit shift and add).  So a sample is four ALU ops to its place, one
// LDS read and a running 16-bit sum, and a second scan carries the sum across lanes.  Outputs leave
// as two 16-byte stores per lane.
__device__ __forceinline__ void merge_step(const MergeLds& W, uint32_t kw, uint32_t pS, uint32_t pM, uint32_t pL,
                                           uint32_t& carry, int16_t* __restrict__ out, uint32_t t, uint32_t n, bool full)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint8_t* wb = reinterpret_cast<const uint8_t*>(&W);
    constexpr uint32_t pZ = (uint32_t)__builtin_offsetof(MergeLds, zero);
    // places are below sizeof(MergeLds) < 2^16
    uint32_t plo = pZ | (pS << 16), phi = pM | (pL << 16);
    uint32_t acc = 0;  // the running sum (its low 16 bits)
    uint32_t w[8];     // running sums, two 16-bit samples per word
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t a[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int m = 2 * k + h;
            const uint32_t c = __builtin_amdgcn_ubfe(kw, 2 * m, 2);
            const uint32_t at = __builtin_amdgcn_perm(phi, plo, c * 0x0202u + 0x0C0C0100u);
            if (m < 15) {
                const uint64_t inc = (uint64_t)2 << (16 * c);
                plo += (uint32_t)inc;
                phi += (uint32_t)(inc >> 32);
            }
            acc += *reinterpret_cast<const uint16_t*>(wb + at);
            a[h] = acc;
        }
        w[k] = __builtin_amdgcn_perm(a[1], a[0], 0x05040100u);  // the two sums' low halves
        if (k & 1) __builtin_amdgcn_sched_barrier(0);  // at most 4 places read ahead (VGPRs)
    }
    acc &= 0xFFFFu;
    const uint32_t incl = wave_incl_sum(acc);
    const uint32_t base = carry + incl - acc;
    carry += readlane_u32(incl, 63);
    const pgn_u16x2 base2 = as_u16x2((base & 0xFFFFu) * 0x00010001u);
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = as_u32(as_u16x2(w[k]) + base2);
    int16_t* dst = out + t + 16u * lane;
    if (full) {
        // the samples are written once: non-temporal stores (they do not displace the streams the
        // other decode kernels are reading from L2; bench-size decode 22.3-22.6 -> 21.8-21.9 ms)
        if (((uintptr_t)dst & 15u) == 0) {
            gst_nt16(dst, make_uint4(w[0], w[1], w[2], w[3]));
            gst_nt16(dst + 8, make_uint4(w[4], w[5], w[6], w[7]));
        } else {
            gst<uint4>(dst, make_uint4(w[0], w[1], w[2], w[3]));
            gst<uint4>(dst + 8, make_uint4(w[4], w[5], w[6], w[7]));
        }
    } else {
        for (uint32_t m = 0; m < 16 && t + 16u * lane + m < n; m++) gst<uint16_t>(dst + m, (uint16_t)(w[m >> 1] >> (16 * (m & 1))));
    }
}

// One step's bookkeeping, computed two steps ahead: the key word, the class counts below this lane,
// the step's totals, the staging ranges of its S / M / class-3 bytes, and the stream counts before it.
struct MergePlan {  // offsets in the intermediate are 32-bit (a chunk's intermediate is < 40 MB)
    uint32_t kw;
    uint32_t excl;        // classes 1 | 2 << 11 | 3 << 22 of the lanes below (exact: at most 1008 each)
    uint32_t ns, nm, nl;  // the step's class counts
    uint32_t sN, mN, lN;  // S nibbles / M bytes / class-3 pairs before the step
    uint32_t nwS, nbM;    // S dwords, M 16-byte blocks from the 16-byte blocks holding the step's first bytes
};
// A step's stream bytes in flight (loaded two steps before they are staged)
struct MergeBytes {
    uint4 vM;
    uint32_t vS, lb, hb;
};

// The merge of the steps [t0, t1) of a chunk (t0 a multiple of kSplitStep, t1 = n or one), given
// the class counts of the samples before t0 (sN0 / mN0 / lN0) and the running sum there (carry, in
// and out); *lEnd receives the class-3 count through t1.  c5_merge_wave is the whole chunk in one
// call; dec_merge_lb_kernel gives the ranges of one chunk to single-wave workgroups.
// Software pipeline (one wave per chunk): a step's key word is loaded kMergeAhead + 2 steps ahead,
// its plan made and its S / M / class-3 bytes loaded kMergeAhead steps ahead (kMergeAhead = 2: two
// register sets, the loop unrolled by two).  Measured (tools/gpu_ab_kern.sh, 20,000 chunks): two
// steps ahead is no faster than one (1.54 vs 1.50 ms; the merge is issue-bound), and at
// six waves per SIMD it spills; so one.  Plan offsets are 32-bit (fewer scalar instructions).
#ifndef PGN_MERGE_AHEAD
#define PGN_MERGE_AHEAD 1
#endif
constexpr uint32_t kMergeAhead = PGN_MERGE_AHEAD;
static_assert(kMergeAhead == 1 || kMergeAhead == 2, "merge lookahead");
template <bool C4 = false>
__device__ __forceinline__ int c5_merge_range(const uint8_t* __restrict__ in, uint64_t total, uint64_t dS, uint64_t dM,
                                              uint64_t dLl, int16_t* __restrict__ out, uint32_t n, uint32_t t0,
                                              uint32_t t1, uint64_t sN0, uint64_t mN0, uint64_t lN0, uint32_t& carry,
                                              uint64_t* lEnd, MergeLds& W)
{
    using CO = ClassOffsets<C4>;
    const uint32_t lane = (uint32_t)lane_id();
    // stream starts, 32-bit: an intermediate is below 2^31 bytes (inter_cap), the key bytes below
    // 2^22 and the decoded sizes sum to at most `total`, so no sum below overflows
    if (total >= 0x80000000ull || dS + dM + dLl > total) return 1;
    const uint32_t tot = (uint32_t)total;
    const uint32_t kl = (n + 3) / 4;
    const uint32_t ps = kl, pm = kl + (uint32_t)dS, pl = pm + (uint32_t)dM, ph = pl + (uint32_t)dLl;
    uint32_t sN = (uint32_t)sN0, mN = (uint32_t)mN0, lN = (uint32_t)lN0;  // before the next step to plan (wave-uniform)
    if (lane < 16) W.zero[lane] = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {  // the S table: byte -> two entries
        const uint32_t bt = 4 * lane + q;
        W.nib[bt] = (uint32_t)zz_dec16((uint16_t)((bt & 15u) + CO::o1)) |
                    ((uint32_t)zz_dec16((uint16_t)((bt >> 4) + CO::o1)) << 16);
    }
    // the key word of the step at t (codes past the signal's end are not samples)
    auto key_word = [&](uint32_t t) -> uint32_t {
        const bool full = t + kSplitStep <= n;
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        const uint32_t kb0 = t >> 2;
        uint32_t kw = 0;
        if (4u * lane + 4u <= nK) {
            kw = ld32u(in + kb0 + 4u * lane);
        } else {
            for (uint32_t b = 4u * lane; b < nK; b++) kw |= (uint32_t)gb(in + kb0 + b) << (8u * (b - 4u * lane));
        }
        if (!full) {
            const uint32_t first = 16u * lane, nv = (n - t) > first ? (n - t) - first : 0u;
            if (nv < 16) kw &= (1u << (2u * nv)) - 1u;
        }
        return kw;
    };
    // the plan of step t from its key word (the counts advance past it); false if the step reads
    // past `total` (the reference's UB)
    auto plan = [&](uint32_t t, uint32_t kw, MergePlan& pn) -> bool {
        const uint32_t nK = t + kSplitStep <= n ? kSplitStep / 4 : (n - t + 3) / 4;
        if ((t >> 2) + nK > tot) return false;
        const uint32_t lo = kw & 0x55555555u, hi = (kw >> 1) & 0x55555555u;
        const uint32_t pc = (uint32_t)__builtin_popcount(lo & ~hi) | ((uint32_t)__builtin_popcount(hi & ~lo) << 11) |
                            ((uint32_t)__builtin_popcount(lo & hi) << 22);
        const uint32_t inc = wave_incl_sum(pc);
        pn.kw = kw;
        pn.excl = inc - pc;
        // field 3 has 10 bits: rebuild its total from the last lane (the split's wrap rule)
        const uint32_t e63 = readlane_u32(pn.excl, 63), p63 = readlane_u32(pc, 63);
        const uint32_t t12 = readlane_u32(inc, 63);
        pn.ns = t12 & 0x7FFu;
        pn.nm = (t12 >> 11) & 0x7FFu;
        pn.nl = (e63 >> 22) + (p63 >> 22);
        if (ps + ((sN + pn.ns + 1) >> 1) > tot || pm + mN + pn.nm > tot || pl + lN + pn.nl > tot || ph + lN + pn.nl > tot)
            return false;
        const uint32_t aS = ps + (sN >> 1), aM = pm + mN;
        pn.nwS = ((ps + ((sN + pn.ns + 1) >> 1)) - (aS & ~15u) + 3) >> 2;
        pn.nbM = (aM + pn.nm - (aM & ~15u) + 15) >> 4;
        pn.sN = sN;
        pn.mN = mN;
        pn.lN = lN;
        sN += pn.ns;
        mN += pn.nm;
        lN += pn.nl;
        return true;
    };
    auto load_stage = [&](const MergePlan& pn, MergeBytes& B) {
        const uint32_t aS0 = (ps + (pn.sN >> 1)) & ~15u, aM0 = (pm + pn.mN) & ~15u;
        if (lane < pn.nwS) B.vS = gld<uint32_t>(in + aS0 + 4u * lane);
        if (lane < pn.nbM) B.vM = gld<uint4>(in + aM0 + 16u * lane);
        if (lane < pn.nl) {
            B.lb = gb(in + pl + pn.lN + lane);
            B.hb = gb(in + ph + pn.lN + lane);
        }
    };
    if (t0 >= t1) {
        *lEnd = lN;
        return 0;
    }
    const uint32_t nsteps = (t1 - t0 + kSplitStep - 1) / kSplitStep;
    auto tof = [&](uint32_t j) { return t0 + j * kSplitStep; };
    // prologue: the plans and bytes of steps 0 .. kMergeAhead - 1, the key words of the next two
    constexpr uint32_t D = kMergeAhead;
    MergePlan P0, P1;
    MergeBytes B0, B1;
    B0.vM = B1.vM = make_uint4(0, 0, 0, 0);
    B0.vS = B1.vS = B0.lb = B1.lb = B0.hb = B1.hb = 0;
    if (!plan(tof(0), key_word(tof(0)), P0)) return 1;
    load_stage(P0, B0);
    if (D == 2 && nsteps > 1) {
        if (!plan(tof(1), key_word(tof(1)), P1)) return 1;
        load_stage(P1, B1);
    }
    uint32_t kwN1 = nsteps > D ? key_word(tof(D)) : 0u;          // the next plan's key word
    uint32_t kwN2 = nsteps > D + 1 ? key_word(tof(D + 1)) : 0u;  // and the one after it
    lds_sync();
    // step j from plan P / bytes B; then plan step j + D into P and load its bytes into B
    auto body = [&](uint32_t j, MergePlan& P, MergeBytes& B) -> bool {
        const uint32_t t = tof(j);
        const bool full = t + kSplitStep <= n;
        // ---- this step's bytes into the window: S by table, M and class 3 by arithmetic
        // S: four bytes (eight entries) per lane, so the step's ~170 S bytes take four table reads
        // per lane instead of sixteen on a quarter of the lanes
        const uint32_t eM = 8u * P.nwS, eL = eM + 16u * P.nbM;
        const uint32_t aS = ps + (P.sN >> 1), aM = pm + P.mN, aS0 = aS & ~15u, aM0 = aM & ~15u;
        {
            constexpr uint32_t add2 = CO::o2 * 0x00010001u;
            auto put_s4 = [&](uint32_t b, uint32_t v) {
                *(uint4*)(W.V + 8u * b) = make_uint4(W.nib[v & 0xFFu], W.nib[(v >> 8) & 0xFFu], W.nib[(v >> 16) & 0xFFu],
                                                     W.nib[v >> 24]);
            };
            if (lane < P.nwS) put_s4(lane, B.vS);
            if (lane < P.nbM) put_bytes16(W.V + eM + 16u * lane, B.vM, add2);
            if (lane < P.nl) W.V[eL + lane] = zz_dec16((uint16_t)((B.lb | (B.hb << 8)) + CO::o3));
            for (uint32_t b = lane + 64; b < P.nwS; b += 64) put_s4(b, gld<uint32_t>(in + aS0 + 4u * b));
            for (uint32_t b = lane + 64; b < P.nbM; b += 64) put_bytes16(W.V + eM + 16u * b, gld<uint4>(in + aM0 + 16u * b), add2);
            for (uint32_t i = lane + 64; i < P.nl; i += 64)
                W.V[eL + i] = zz_dec16((uint16_t)(((uint32_t)gb(in + pl + P.lN + i) | ((uint32_t)gb(in + ph + P.lN + i) << 8)) + CO::o3));
        }
        lds_sync();
        // LDS byte places of my first value of each class
        constexpr uint32_t offV = (uint32_t)__builtin_offsetof(MergeLds, V);
        const uint32_t pS = offV + 2u * ((2 * (aS - aS0) + (P.sN & 1u)) + (P.excl & 0x7FFu));
        const uint32_t pM = offV + 2u * (eM + (aM - aM0) + ((P.excl >> 11) & 0x7FFu));
        const uint32_t pL = offV + 2u * (eL + (P.excl >> 22));
        const uint32_t kw = P.kw;
        // ---- step j + D: its plan (key word loaded two steps ago), its bytes in flight for D steps
        if (j + D < nsteps) {
            if (!plan(tof(j + D), kwN1, P)) return false;
            load_stage(P, B);
        }
        kwN1 = kwN2;
        if (j + D + 2 < nsteps) kwN2 = key_word(tof(j + D + 2));
        merge_step(W, kw, pS, pM, pL, carry, out, t, n, full);
        lds_sync();
        return true;
    };
    if (D == 1) {
        for (uint32_t j = 0; j < nsteps; j++)
            if (!body(j, P0, B0)) return 1;
    } else {
        for (uint32_t j = 0; j < nsteps; j += 2) {
            if (!body(j, P0, B0)) return 1;
            if (j + 1 >= nsteps) break;
            if (!body(j + 1, P1, B1)) return 1;
        }
    }
    *lEnd = lN;
    return 0;
}

template <bool C4 = false>
__device__ __forceinline__ int c5_merge_wave(const uint8_t* __restrict__ in, uint64_t total, uint64_t dS, uint64_t dM,
                                             uint64_t dLl, int16_t* __restrict__ out, uint32_t n, uint64_t* consumed,
                                             MergeLds& W)
{
    const uint64_t kl = ((uint64_t)n + 3) / 4;
    uint32_t carry = 0;
    uint64_t lN = 0;
    const int bad = c5_merge_range<C4>(in, total, dS, dM, dLl, out, n, 0u, n, 0, 0, 0, carry, &lN, W);
    if (bad) return bad;
    *consumed = kl + dS + dM + dLl + lN;
    return 0;
}

// Sum (mod 2^16) of the deltas the samples of a range decode to -- order-free, so it is a plain
// reduction over the range's stretches of the S / M / class-3 streams: S nibbles [s0, s1) at ps
// (low nibble first), M bytes [m0, m1) at pm, class-3 pairs [l0, l1) at pl / ph.  Wave-uniform.
template <bool C4 = false>
__device__ inline uint32_t c5_range_delta_sum(const uint8_t* __restrict__ in, uint64_t ps, uint64_t pm, uint64_t pl,
                                              uint64_t ph, uint64_t s0, uint64_t s1, uint64_t m0, uint64_t m1,
                                              uint64_t l0, uint64_t l1)
{
    using CO = ClassOffsets<C4>;
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t acc = 0;
    // S: bytes [s0 / 2, (s1 + 1) / 2), nibble i of the range in byte i / 2
    {
        const uint64_t b0 = ps + (s0 >> 1), b1 = ps + ((s1 + 1) >> 1);
        for (uint64_t bb = (b0 & ~(uint64_t)15) + 16u * lane; bb < b1; bb += 4096) {
          uint4 vv[4];
#pragma unroll
          for (int u = 0; u < 4; u++) vv[u] = bb + 1024u * u < b1 ? gld<uint4>(in + bb + 1024u * u) : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const uint64_t blk = bb + 1024u * u;
            if (blk >= b1) break;
            const uint4 v = vv[u];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint64_t nib0 = 2 * (blk + j - ps);  // this byte's low nibble index
                const uint32_t by = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if (nib0 >= s0 && nib0 < s1) acc += zz_dec16((uint16_t)((by & 15u) + CO::o1));
                if (nib0 + 1 >= s0 && nib0 + 1 < s1) acc += zz_dec16((uint16_t)((by >> 4) + CO::o1));
            }
          }
        }
    }
    {
        const uint64_t b0 = pm + m0, b1 = pm + m1;
        for (uint64_t bb = (b0 & ~(uint64_t)15) + 16u * lane; bb < b1; bb += 4096) {
            uint4 vv[4];
#pragma unroll
            for (int u = 0; u < 4; u++) vv[u] = bb + 1024u * u < b1 ? gld<uint4>(in + bb + 1024u * u) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t blk = bb + 1024u * u;
                const uint32_t w[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const uint64_t p = blk + j;
                    if (p >= b0 && p < b1) acc += zz_dec16((uint16_t)(((w[j >> 2] >> (8 * (j & 3))) & 0xFFu) + CO::o2));
                }
            }
        }
    }
    for (uint64_t i = l0 + lane; i < l1; i += 64)
        acc += zz_dec16((uint16_t)(((uint32_t)gb(in + pl + i) | ((uint32_t)gb(in + ph + i) << 8)) + CO::o3));
    return wave_sum(acc & 0xFFFFu) & 0xFFFFu;
}

// Class counts (S, M, class 3) of the samples in [t0, t1) from their keys (2 bits per sample, 16
// samples per key word; codes past n are not samples), wave-uniform.
__device__ inline void c5_class_counts(const uint8_t* __restrict__ in, uint32_t n, uint32_t t0, uint32_t t1,
                                       uint32_t& cS, uint32_t& cM, uint32_t& cL)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t s = 0, m = 0, l = 0;
    // four 1,024-sample steps per trip, their key loads issued together
    for (uint32_t tb = t0; tb < t1; tb += 4096u) {
        uint32_t kw[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + 1024u * u + 16u * lane;
            kw[u] = 0;
            if (t < t1) {
                const uint32_t nK = (n - t + 3) / 4 < 4u ? (n - t + 3) / 4 : 4u;
                if (nK == 4) {
                    kw[u] = ld32u(in + (t >> 2));
                } else {
                    for (uint32_t b = 0; b < nK; b++) kw[u] |= (uint32_t)gb(in + (t >> 2) + b) << (8u * b);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + 1024u * u + 16u * lane;
            uint32_t k = kw[u];
            if (t >= t1) k = 0;
            else if (n - t < 16) k &= (1u << (2u * (n - t))) - 1u;
            const uint32_t lo = k & 0x55555555u, hi = (k >> 1) & 0x55555555u;
            s += (uint32_t)__builtin_popcount(lo & ~hi);
            m += (uint32_t)__builtin_popcount(hi & ~lo);
            l += (uint32_t)__builtin_popcount(lo & hi);
        }
    }
    cS = wave_sum(s);
    cM = wave_sum(m);
    cL = wave_sum(l);
}

}  // namespace pgn
