// pgn_c5.h -- C5 ("N01") split and merge on one wave.
//
// Split = svb16::encode_scalar_N01<int16_t, /*delta*/true, /*zigzag*/true> (pgnano/svb16/C5.hpp:57-152)
// Merge = svb16::decode_scalar_N01 (C5.hpp:173-257) as driven by decode_N01 (C5.hpp:260-275) and
//         decompress_signal_N01's consumed-bytes check (C5.hpp:669-677).
//
// The reference walks the samples serially; here a wave takes 1024 samples per step (16 per lane,
// four key bytes per lane), classifies them, and places every S/M/L value with one wave prefix sum
// of the per-lane class counts.  Stream bytes are assembled in LDS bit windows and leave as aligned
// dword stores; the wrapping 16-bit delta is undone with a wave prefix sum.
#pragma once
#include "pgn_wave.h"

namespace pgn {

__device__ __forceinline__ uint16_t zz_enc16(uint16_t v) { return (uint16_t)((uint16_t)(v + v) ^ (uint16_t)((int16_t)v >> 15)); }
__device__ __forceinline__ uint16_t zz_dec16(uint16_t v) { return (uint16_t)((v >> 1) ^ (uint16_t)(0u - (v & 1u))); }

struct C5Streams {
    uint8_t *K, *S, *M, *Ll, *Lh;
};

// ---------------------------------------------------------------------------------------------
// LDS bit window: bits [base*8, ...) of an output byte stream are assembled by OR-ing lane pieces
// into words, then complete words are flushed to global memory (dword aligned: base % 4 == 0).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void win_or64(uint32_t* win, uint32_t bitpos, uint64_t v, uint32_t nbits)
{
    if (nbits == 0) return;
    const uint32_t w = bitpos >> 5, sh = bitpos & 31;
    atomicOr(&win[w], (uint32_t)(v << sh));
    if (sh + nbits > 32) atomicOr(&win[w + 1], (uint32_t)((v << sh) >> 32));
    if (sh + nbits > 64) atomicOr(&win[w + 2], (uint32_t)(v >> (64 - sh)));
}

// flush the complete words of a window holding `bits` bits; returns the carried partial word.
// Caller: lds_sync() before; afterwards the window is zero except word 0 = carry.
__device__ __forceinline__ void win_flush(uint32_t* win, uint32_t nwords, uint32_t bits, uint8_t* out)
{
    const int lane = lane_id();
    const uint32_t complete = bits >> 5;
    for (uint32_t w = (uint32_t)lane; w < complete; w += 64) gst<uint32_t>(out + 4 * w, win[w]);
    const uint32_t carry = win[complete];
    lds_sync();
    for (uint32_t w = (uint32_t)lane; w < nwords; w += 64) win[w] = (w == 0) ? carry : 0u;
    lds_sync();
}

constexpr uint32_t kSplitStep = 1024;
constexpr uint32_t kWinS = 132, kWinB = 264;  // words

struct SplitLds {
    uint32_t S[kWinS];
    uint32_t M[kWinB];
    uint32_t Ll[kWinB];
    uint32_t Lh[kWinB];
};

// sizes[5] = {keys, S, M, Llow, Lhigh} bytes.
__device__ __noinline__ void c5_split_wave(const int16_t* __restrict__ x, uint32_t n, const C5Streams& st, uint32_t sizes[5],
                                     SplitLds& W)
{
    const int lane = lane_id();
    if (n == 0) {
        for (int i = 0; i < 5; i++) sizes[i] = 0;
        return;
    }
    for (uint32_t w = (uint32_t)lane; w < kWinB; w += 64) {
        if (w < kWinS) W.S[w] = 0;
        W.M[w] = 0;
        W.Ll[w] = 0;
        W.Lh[w] = 0;
    }
    lds_sync();
    // stream positions: totals so far; window bases (bytes, multiple of 4) in each stream
    uint32_t sTot = 0, mTot = 0, lTot = 0;  // S in nibbles
    uint32_t sBase = 0, mBase = 0, lBase = 0;
    uint16_t prevStep = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const uint32_t i0 = t + 16u * (uint32_t)lane;
        uint16_t xs[16];
        if (i0 + 16 <= n) {
            const uint4 a = gld<uint4>(x + i0), b = gld<uint4>(x + i0 + 8);
            __builtin_memcpy(xs, &a, 16);
            __builtin_memcpy(xs + 8, &b, 16);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) xs[j] = (i0 + j < n) ? gld<uint16_t>(x + i0 + j) : (uint16_t)0;
        }
        const uint16_t prevLane = (uint16_t)__shfl_up((int)xs[15], 1, 64);
        uint16_t prev = (lane == 0) ? prevStep : prevLane;
        uint32_t key = 0, ns = 0, nm = 0, nl = 0;
        uint64_t sAcc = 0;        // up to 16 nibbles
        uint64_t mAcc0 = 0, mAcc1 = 0, lAcc0 = 0, lAcc1 = 0, hAcc0 = 0, hAcc1 = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint16_t v = zz_enc16((uint16_t)(xs[j] - prev));
            prev = xs[j];
            const bool in = (i0 + j < n);
            const uint32_t c = !in ? 0u : (v == 0 ? 0u : (v <= 16 ? 1u : (v <= 272 ? 2u : 3u)));
            key |= c << (2 * j);
            if (c == 1) {
                sAcc |= (uint64_t)(v - 1) << (4 * ns);
                ns++;
            } else if (c == 2) {
                const uint64_t b = (uint64_t)(uint8_t)(v - 17);
                if (nm < 8) mAcc0 |= b << (8 * nm); else mAcc1 |= b << (8 * (nm - 8));
                nm++;
            } else if (c == 3) {
                const uint32_t w = (uint32_t)v - 273u;
                const uint64_t lo = w & 0xFF, hi = w >> 8;
                if (nl < 8) { lAcc0 |= lo << (8 * nl); hAcc0 |= hi << (8 * nl); }
                else { lAcc1 |= lo << (8 * (nl - 8)); hAcc1 |= hi << (8 * (nl - 8)); }
                nl++;
            }
        }
        const uint64_t packed = (uint64_t)ns | ((uint64_t)nm << 16) | ((uint64_t)nl << 32);
        const uint64_t incl = wave_incl_sum64(packed);
        const uint64_t excl = incl - packed;
        const uint64_t tot = readlane_u64(incl, 63);
        if (i0 < n) gst<uint32_t>(st.K + (i0 >> 2), key);
        // window-relative bit positions
        const uint32_t sBit = 4u * (sTot - 2u * sBase + (uint32_t)(excl & 0xFFFF));
        const uint32_t mBit = 8u * (mTot - mBase + (uint32_t)((excl >> 16) & 0xFFFF));
        const uint32_t lBit = 8u * (lTot - lBase + (uint32_t)(excl >> 32));
        win_or64(W.S, sBit, sAcc, 4 * ns);
        win_or64(W.M, mBit, mAcc0, 8 * (nm < 8 ? nm : 8));
        if (nm > 8) win_or64(W.M, mBit + 64, mAcc1, 8 * (nm - 8));
        win_or64(W.Ll, lBit, lAcc0, 8 * (nl < 8 ? nl : 8));
        win_or64(W.Lh, lBit, hAcc0, 8 * (nl < 8 ? nl : 8));
        if (nl > 8) {
            win_or64(W.Ll, lBit + 64, lAcc1, 8 * (nl - 8));
            win_or64(W.Lh, lBit + 64, hAcc1, 8 * (nl - 8));
        }
        sTot += (uint32_t)(tot & 0xFFFF);
        mTot += (uint32_t)((tot >> 16) & 0xFFFF);
        lTot += (uint32_t)(tot >> 32);
        lds_sync();
        // flush complete words (dword aligned in every stream)
        const uint32_t sBits = 4u * (sTot - 2u * sBase), mBits = 8u * (mTot - mBase), lBits = 8u * (lTot - lBase);
        win_flush(W.S, kWinS, sBits, st.S + sBase);
        win_flush(W.M, kWinB, mBits, st.M + mBase);
        win_flush(W.Ll, kWinB, lBits, st.Ll + lBase);
        win_flush(W.Lh, kWinB, lBits, st.Lh + lBase);
        sBase += 4u * (sBits >> 5);
        mBase += 4u * (mBits >> 5);
        lBase += 4u * (lBits >> 5);
        prevStep = (uint16_t)readlane_u32(xs[15], 63);
    }
    // tails: the carried partial words (a trailing odd nibble leaves its high half zero)
    if (lane == 0) {
        gst<uint32_t>(st.S + sBase, W.S[0]);
        gst<uint32_t>(st.M + mBase, W.M[0]);
        gst<uint32_t>(st.Ll + lBase, W.Ll[0]);
        gst<uint32_t>(st.Lh + lBase, W.Lh[0]);
    }
    sizes[0] = (n + 3) / 4;
    sizes[1] = (sTot + 1) / 2;
    sizes[2] = mTot;
    sizes[3] = lTot;
    sizes[4] = lTot;
}

// Merge over the reference's concatenated intermediate buffer (see oracle c5_merge): stream starts at
// keys_length = ceil(n/4), then +dS, +dM, +dLl; a read past `total` is the reference's UB -> error.
// `in` must stay readable 16 bytes past `total` (scratch padding).  Returns 0 ok, 1 out-of-bounds;
// *consumed = one past the last Lhigh byte.
__device__ __noinline__ int c5_merge_wave(const uint8_t* __restrict__ in, uint64_t total, uint64_t dS, uint64_t dM,
                                    uint64_t dLl, int16_t* __restrict__ out, uint32_t n, uint64_t* consumed)
{
    const int lane = lane_id();
    const uint64_t kl = ((uint64_t)n + 3) / 4;
    const uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    uint64_t sN = 0, mN = 0, lN = 0;
    uint16_t carry = 0;
    bool bad = false;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const uint32_t i0 = t + 16u * (uint32_t)lane;
        const uint32_t nv = (i0 >= n) ? 0u : ((n - i0) < 16u ? n - i0 : 16u);  // valid samples of this lane
        uint32_t key = 0;
        if (nv) {
            const uint64_t kb = i0 >> 2;
            if (kb + ((nv + 3) >> 2) <= total) key = ld32u(in + kb);
            else bad = true;
            if (nv < 16) key &= (1u << (2 * nv)) - 1;  // codes past the end are ignored
        }
        // class counts from the 2-bit codes
        const uint32_t lo = key & 0x55555555u, hi = (key >> 1) & 0x55555555u;
        const uint32_t m1 = lo & ~hi, m2 = hi & ~lo, m3 = lo & hi;
        const uint32_t ns = __builtin_popcount(m1), nm = __builtin_popcount(m2), nl = __builtin_popcount(m3);
        const uint64_t packed = (uint64_t)ns | ((uint64_t)nm << 16) | ((uint64_t)nl << 32);
        const uint64_t incl = wave_incl_sum64(packed);
        const uint64_t excl = incl - packed;
        const uint64_t tot = readlane_u64(incl, 63);
        const uint64_t sq = sN + (excl & 0xFFFF), mq = mN + ((excl >> 16) & 0xFFFF), lq = lN + (excl >> 32);
        // gather this lane's contiguous runs
        uint64_t sv = 0, sv2 = 0, mv0 = 0, mv1 = 0, lv0 = 0, lv1 = 0, hv0 = 0, hv1 = 0;
        if (ns) {
            const uint64_t b0 = ps + (sq >> 1), bEnd = ps + ((sq + ns + 1) >> 1);
            if (bEnd <= total) { sv = ld64u(in + b0); sv2 = gb(in + b0 + 8); }
            else bad = true;
        }
        if (nm) {
            if (pm + mq + nm <= total) { mv0 = ld64u(in + pm + mq); mv1 = ld64u(in + pm + mq + 8); }
            else bad = true;
        }
        if (nl) {
            if (pl + lq + nl <= total && ph + lq + nl <= total) {
                lv0 = ld64u(in + pl + lq); lv1 = ld64u(in + pl + lq + 8);
                hv0 = ld64u(in + ph + lq); hv1 = ld64u(in + ph + lq + 8);
            } else {
                bad = true;
            }
        }
        // nibble stream aligned to this lane's first nibble
        const uint32_t sh = (uint32_t)(sq & 1) * 4;
        uint64_t sNib = (sv >> sh) | (sh ? (sv2 << (64 - sh)) : 0);
        uint32_t is = 0, im = 0, il = 0;
        uint16_t d[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t c = (key >> (2 * j)) & 3u;
            uint16_t v = 0;
            if (c == 1) {
                v = (uint16_t)(((sNib >> (4 * is)) & 15u) + 1u);
                is++;
            } else if (c == 2) {
                v = (uint16_t)(((im < 8 ? (mv0 >> (8 * im)) : (mv1 >> (8 * (im - 8)))) & 0xFF) + 17u);
                im++;
            } else if (c == 3) {
                const uint32_t l8 = (uint32_t)((il < 8 ? (lv0 >> (8 * il)) : (lv1 >> (8 * (il - 8)))) & 0xFF);
                const uint32_t h8 = (uint32_t)((il < 8 ? (hv0 >> (8 * il)) : (hv1 >> (8 * (il - 8)))) & 0xFF);
                v = (uint16_t)((h8 << 8) + l8 + 273u);
                il++;
            }
            d[j] = ((uint32_t)j < nv) ? zz_dec16(v) : (uint16_t)0;
        }
        uint16_t run[16];
        uint16_t acc = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) { acc = (uint16_t)(acc + d[j]); run[j] = acc; }
        const uint32_t lincl = wave_incl_sum(acc);
        const uint16_t base = (uint16_t)(carry + (uint16_t)(lincl - acc));
        if (nv == 16) {
            uint16_t o[16];
#pragma unroll
            for (int j = 0; j < 16; j++) o[j] = (uint16_t)(base + run[j]);
            uint4 a, b;
            __builtin_memcpy(&a, o, 16);
            __builtin_memcpy(&b, o + 8, 16);
            gst<uint4>(out + i0, a);
            gst<uint4>(out + i0 + 8, b);
        } else {
            for (uint32_t j = 0; j < nv; j++) gst<uint16_t>(out + i0 + j, (uint16_t)(base + run[j]));
        }
        carry = (uint16_t)(carry + (uint16_t)readlane_u32(lincl, 63));
        sN += tot & 0xFFFF;
        mN += (tot >> 16) & 0xFFFF;
        lN += tot >> 32;
    }
    *consumed = ph + lN;
    return ballot(bad) ? 1 : 0;
}

}  // namespace pgn
