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
// Split.  A step is 1024 samples; sub-step k gives lane l sample t + 64k + l.  The class of every
// sample becomes three wave ballots; a value's place in its stream is the stream's fill plus the
// number of same-class lanes below it (mbcnt), so each lane writes its byte straight into an LDS
// window.  Keys are OR-ed across lane quads with DPP.  After a step, complete 16-byte blocks of
// each window go to HBM as aligned 16-byte stores and the tail moves to the window front.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kSplitStep = 1024;
constexpr uint32_t kWinBytes = 1088;  // 31 carried nibbles + 1024 new, rounded up to 16

struct SplitLds {
    alignas(16) uint8_t S[kWinBytes];  // one byte per nibble
    alignas(16) uint8_t M[kWinBytes];
    alignas(16) uint8_t L[kWinBytes];
    alignas(16) uint8_t H[kWinBytes];
    alignas(16) uint8_t K[kSplitStep / 4];
};

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

// One 1024-sample step (Full: every sample of the step exists).  Per sub-step: three compares give
// the class ballots (classes combined in scalar registers), each class's bytes go to its window
// at fill + mbcnt rank under that class's exec mask (class 3 is rare and usually skipped whole),
// and the quad-OR-ed key byte is written by all four lanes of a quad (same byte, no masking).
template <bool Full>
__device__ __forceinline__ void split_step(const int16_t* __restrict__ x, uint32_t n, uint32_t t, SplitLds& W,
                                           uint32_t& fS, uint32_t& fM, uint32_t& fL, uint32_t& prevX)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t xv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // a partial step re-reads the last sample (masked below)
        const uint32_t i = t + 64u * (uint32_t)k + lane;
        xv[k] = (uint32_t)gld<uint16_t>(x + (Full ? i : (i < n ? i : n - 1)));
    }
    const uint32_t ksh = 2u * (lane & 3u);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t cur = xv[k];
        uint32_t prv = dpp<kDppWaveShr1>(cur);
        prv = (lane == 0) ? prevX : prv;
        prevX = readlane_u32(cur, 63);
        const uint32_t v = zz_enc16((uint16_t)(cur - prv));
        const bool valid = Full || (t + 64u * (uint32_t)k + lane < n);
        const bool nz = valid && v != 0, gt16 = v > 16, gt272 = v > 272;
        const uint64_t bnz = ballot(nz), b16 = ballot(gt16), b272 = ballot(gt272);
        const uint64_t b1 = bnz & ~b16, b2 = bnz & b16 & ~b272, b3 = bnz & b272;
        if (nz && !gt16) W.S[fS + mbcnt(b1)] = (uint8_t)(v - 1u);
        if (nz && gt16 && !gt272) W.M[fM + mbcnt(b2)] = (uint8_t)(v - 17u);
        if (b3) {
            if (nz && gt272) {
                const uint32_t w = v - 273u, r = fL + mbcnt(b3);
                W.L[r] = (uint8_t)w;
                W.H[r] = (uint8_t)(w >> 8);
            }
        }
        fS += (uint32_t)__builtin_popcountll(b1);
        fM += (uint32_t)__builtin_popcountll(b2);
        fL += (uint32_t)__builtin_popcountll(b3);
        const uint32_t c = (uint32_t)nz + (uint32_t)(nz && gt16) + (uint32_t)(nz && gt272);
        uint32_t kb = c << ksh;
        kb |= dpp<kDppQuadSwap1>(kb);
        kb |= dpp<kDppQuadSwap2>(kb);
        W.K[16u * (uint32_t)k + (lane >> 2)] = (uint8_t)kb;
    }
}

// sizes[5] = {keys, S, M, Llow, Lhigh} bytes.
__device__ __forceinline__ void c5_split_wave(const int16_t* __restrict__ x, uint32_t n, const C5Streams& st, uint32_t sizes[5],
                                              SplitLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t fS = 0, fM = 0, fL = 0, fH = 0;  // window fills (S in nibbles)
    uint32_t gS = 0, gM = 0, gL = 0, gH = 0;  // bytes already in HBM
    uint32_t prevX = 0;                       // last sample of the previous sub-step (wave-uniform)
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        if (full) split_step<true>(x, n, t, W, fS, fM, fL, prevX);
        else split_step<false>(x, n, t, W, fS, fM, fL, prevX);
        fH = fL;
        lds_sync();
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        uint8_t* kout = st.K + (t >> 2);
        if (4u * lane + 4u <= nK) gst<uint32_t>(kout + 4u * lane, *(const uint32_t*)(W.K + 4u * lane));
        else for (uint32_t b = 4u * lane; b < nK; b++) gst<uint8_t>(kout + b, W.K[b]);
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
// Merge over the reference's concatenated intermediate buffer (see oracle c5_merge): stream starts at
// keys_length = ceil(n/4), then +dS, +dM, +dLl; a read past `total` is the reference's UB -> error.
// Same lane mapping as the split (sub-step k gives lane l sample t + 64k + l).  Per step the class
// counts come from the key bytes, the step's S/M/L bytes are staged into LDS with 16-byte loads,
// each lane then reads its byte at the class fill plus its mbcnt rank, and the 16-bit delta sum is
// a DPP wave scan.  `in` must stay readable 16 bytes past `total` (scratch padding).
// Returns 0 ok, 1 out-of-bounds; *consumed = one past the last Lhigh byte.
// ---------------------------------------------------------------------------------------------
struct MergeLds {
    alignas(16) uint8_t K[kSplitStep / 4];
    alignas(16) uint8_t S[528];   // 513 bytes of nibbles + alignment
    alignas(16) uint8_t M[1040];  // 1024 + alignment
    alignas(16) uint8_t L[1040];
    alignas(16) uint8_t H[1040];
};

// stage bytes [a, a + len) of `in` (len <= cap - 15) into W; returns the window's first address
__device__ __forceinline__ uint64_t stage_bytes(uint8_t* W, const uint8_t* in, uint64_t a, uint32_t len)
{
    const uint64_t a0 = a & ~(uint64_t)15;
    const uint32_t nblk = (uint32_t)((a + len - a0 + 15) >> 4);
    for (uint32_t b = (uint32_t)lane_id(); b < nblk; b += 64) *(uint4*)(W + 16u * b) = gld<uint4>(in + a0 + 16u * b);
    return a0;
}

__device__ __forceinline__ int c5_merge_wave(const uint8_t* __restrict__ in, uint64_t total, uint64_t dS, uint64_t dM,
                                             uint64_t dLl, int16_t* __restrict__ out, uint32_t n, uint64_t* consumed)
{
    __shared__ MergeLds W;
    const uint32_t lane = (uint32_t)lane_id();
    const uint64_t kl = ((uint64_t)n + 3) / 4;
    const uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    uint64_t sN = 0, mN = 0, lN = 0;  // nibbles / bytes consumed so far (wave-uniform)
    uint32_t carry = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        const uint64_t kb0 = t >> 2;
        if (kb0 + nK > total) return 1;
        uint32_t kw = 0;
        if (4u * lane + 4u <= nK) {
            kw = ld32u(in + kb0 + 4u * lane);
        } else {
            for (uint32_t b = 4u * lane; b < nK; b++) kw |= (uint32_t)gb(in + kb0 + b) << (8u * (b - 4u * lane));
        }
        if (!full) {  // codes past the end of the signal are not samples
            const uint32_t first = 16u * lane, nv = (n - t) > first ? (n - t) - first : 0u;
            if (nv < 16) kw &= (1u << (2u * nv)) - 1u;
        }
        *(uint32_t*)(W.K + 4u * lane) = kw;
        // class counts of the step
        const uint32_t lo = kw & 0x55555555u, hi = (kw >> 1) & 0x55555555u;
        const uint32_t ns = wave_sum((uint32_t)__builtin_popcount(lo & ~hi));
        const uint32_t nm = wave_sum((uint32_t)__builtin_popcount(hi & ~lo));
        const uint32_t nl = wave_sum((uint32_t)__builtin_popcount(lo & hi));
        if (ps + ((sN + ns + 1) >> 1) > total || pm + mN + nm > total || pl + lN + nl > total || ph + lN + nl > total)
            return 1;
        const uint64_t wS = stage_bytes(W.S, in, ps + (sN >> 1), (uint32_t)(((sN + ns + 1) >> 1) - (sN >> 1)));
        const uint64_t wM = stage_bytes(W.M, in, pm + mN, nm);
        const uint64_t wL = stage_bytes(W.L, in, pl + lN, nl);
        const uint64_t wH = stage_bytes(W.H, in, ph + lN, nl);
        lds_sync();
        // window-relative fills: S in nibbles from the window start, M/L in bytes
        uint32_t fS = (uint32_t)(2 * (ps - wS) + sN), fM = (uint32_t)(pm + mN - wM), fL = (uint32_t)(pl + lN - wL);
        const uint32_t dLH = (uint32_t)((ph - wH) - (pl - wL));  // H window offset relative to L's
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t i = t + 64u * (uint32_t)k + lane;
            const uint32_t c = ((uint32_t)W.K[16u * (uint32_t)k + (lane >> 2)] >> (2u * (lane & 3u))) & 3u;
            const uint64_t b1 = ballot(c == 1), b2 = ballot(c == 2), b3 = ballot(c == 3);
            uint32_t v = 0;
            if (c == 1) {
                const uint32_t q = fS + mbcnt(b1);
                v = (((uint32_t)W.S[q >> 1] >> (4u * (q & 1u))) & 15u) + 1u;
            } else if (c == 2) {
                v = (uint32_t)W.M[fM + mbcnt(b2)] + 17u;
            } else if (c == 3) {
                const uint32_t q = fL + mbcnt(b3);
                v = (((uint32_t)W.H[q + dLH] << 8) | (uint32_t)W.L[q]) + 273u;
            }
            fS += (uint32_t)__builtin_popcountll(b1);
            fM += (uint32_t)__builtin_popcountll(b2);
            fL += (uint32_t)__builtin_popcountll(b3);
            const uint32_t incl = wave_incl_sum(zz_dec16((uint16_t)v)) + carry;
            carry = readlane_u32(incl, 63);
            if (full || i < n) gst<uint16_t>(out + i, (uint16_t)incl);
        }
        sN += ns;
        mN += nm;
        lN += nl;
        lds_sync();
    }
    *consumed = ph + lN;
    return 0;
}

}  // namespace pgn
