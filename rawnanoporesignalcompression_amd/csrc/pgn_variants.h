// pgn_variants.h -- split and merge of the other compile-time pgnano variants on one wave
// (pgnano.cpp:70-92 / 105-125 select one with #define COMPRESSOR_*; here they are a runtime codec):
//
//   C2   encode_scalar_lh / decode_scalar_lh       (pgnano/svb16/C2.hpp:52-189): 1-bit keys, the low
//        byte of every sample, the high byte of the samples >= 256
//   C3   encode_scalar_ll_lh / decode_scalar_ll_lh (C3.hpp:53-206): 1-bit keys, low bytes of the small
//        samples, low and high bytes of the big ones
//   VBZ0 encode_scalar_VBZ1 / decode_scalar_VBZ1   (VBZ_0.hpp:60-290): C5's 2-bit classes and offsets,
//        the value as 1 / 2 / 4 nibbles (low first) of one nibble stream after the keys
//
// (C4 is C5's split with the class offsets dropped: pgn_c5.h ClassOffsets; C1 is the svb16 split of
// pgn_vbz.h cut into a keys frame and a data frame.)
//
// Same lane mapping as the C5 and VBZ code: a step is 1024 samples, lane l owns samples
// t + 16l .. t + 16l + 15; the places of its bytes are the stream fills plus DPP wave scans of the
// per-lane class counts.  These variants are not on the benchmark path: bytes leave as single-byte
// stores (nibbles through an LDS window), reads are byte loads.
#pragma once
#include "pgn_vbz.h"

namespace pgn {

// the lane's 16 samples -> zig-zag deltas (prevX: the last sample of the previous step)
template <bool Full>
__device__ __forceinline__ void load_deltas16(const int16_t* __restrict__ x, uint32_t n, uint32_t t, uint32_t& prevX,
                                              uint32_t v[16])
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t i0 = t + 16u * lane;
    uint32_t xv[16];
    if (Full) {
        const uint4 a = gld<uint4>(x + i0), b = gld<uint4>(x + i0 + 8);
        const uint32_t wd[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 8; k++) {
            xv[2 * k] = wd[k] & 0xFFFFu;
            xv[2 * k + 1] = wd[k] >> 16;
        }
    } else {
#pragma unroll
        for (int m = 0; m < 16; m++) xv[m] = (i0 + (uint32_t)m < n) ? (uint32_t)gld<uint16_t>(x + i0 + m) : 0u;
    }
    uint32_t prv = dpp<kDppWaveShr1>(xv[15]);
    prv = (lane == 0) ? prevX : prv;
    prevX = readlane_u32(xv[15], 63);
#pragma unroll
    for (int m = 0; m < 16; m++) {
        v[m] = zz_enc16((uint16_t)(xv[m] - prv));
        prv = xv[m];
    }
}

// the lane's 16 running sums (o[m], acc = o[15]) -> samples: wave scan for the carry, then stores
template <bool Full>
__device__ __forceinline__ void store_samples16(const uint32_t o[16], uint32_t acc, uint32_t& carry,
                                                int16_t* __restrict__ out, uint32_t t, uint32_t n)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t incl = wave_incl_sum(acc);
    const uint32_t base = carry + incl - acc;
    carry += readlane_u32(incl, 63);
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = ((o[2 * k] + base) & 0xFFFFu) | ((o[2 * k + 1] + base) << 16);
    int16_t* dst = out + t + 16u * lane;
    if (Full) {
        gst<uint4>(dst, make_uint4(w[0], w[1], w[2], w[3]));
        gst<uint4>(dst + 8, make_uint4(w[4], w[5], w[6], w[7]));
    } else {
#pragma unroll
        for (int m = 0; m < 16; m++)
            if (t + 16u * lane + (uint32_t)m < n) gst<uint16_t>(dst + m, (uint16_t)(w[m >> 1] >> (16 * (m & 1))));
    }
}

// number of valid samples of the lane in a step
__device__ __forceinline__ uint32_t lane_valid(uint32_t n, uint32_t t)
{
    const uint32_t first = t + 16u * (uint32_t)lane_id();
    return first >= n ? 0u : (n - first < 16u ? n - first : 16u);
}

// ---------------------------------------------------------------------------------------------
// C2 / C3 split: K = 1-bit keys (svb16 layout, bit i%8 of byte i/8: v >= 256), then
//   C2: A = low byte of every sample, H = high bytes of the big samples;
//   C3: A = low bytes of the small samples, B = low bytes of the big ones, H = their high bytes.
// sizes: C2 {keys, A, H}, C3 {keys, A, B, H}.
// ---------------------------------------------------------------------------------------------
template <bool C3>
__device__ __forceinline__ void c23_split_wave(const int16_t* __restrict__ x, uint32_t n, uint8_t* K, uint8_t* A, uint8_t* B,
                                               uint8_t* H, uint32_t sizes[5])
{
    const uint32_t lane = (uint32_t)lane_id();
    for (int s = 0; s < 5; s++) sizes[s] = 0;
    if (n == 0) return;
    const uint32_t nk = svb_key_length(n);
    uint32_t fa = 0, fb = 0, prevX = 0;  // stream fills (wave-uniform)
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        uint32_t v[16];
        if (full) load_deltas16<true>(x, n, t, prevX, v);
        else load_deltas16<false>(x, n, t, prevX, v);
        const uint32_t nv = full ? 16u : lane_valid(n, t);
        uint32_t kw = 0;
#pragma unroll
        for (int m = 0; m < 16; m++) kw |= ((uint32_t)m < nv && v[m] > 255u) ? (1u << m) : 0u;
        const uint32_t kb = (t >> 3) + 2u * lane;
        if (full) {
            gst<uint16_t>(K + kb, (uint16_t)kw);
        } else {
            if (kb < nk) gst<uint8_t>(K + kb, (uint8_t)kw);
            if (kb + 1 < nk) gst<uint8_t>(K + kb + 1, (uint8_t)(kw >> 8));
        }
        const uint32_t nb = (uint32_t)__builtin_popcount(kw), ns = nv - nb;
        const uint32_t p = ns | (nb << 16);
        const uint32_t incl = wave_incl_sum(p);
        const uint32_t tot = readlane_u32(incl, 63), ex = incl - p;
        uint32_t qa = C3 ? fa + (ex & 0xFFFFu) : t + 16u * lane, qb = fb + (ex >> 16);
#pragma unroll
        for (int m = 0; m < 16; m++) {
            if ((uint32_t)m < nv) {
                const bool big = (kw >> m) & 1u;
                if (C3) {
                    if (big) {
                        gst<uint8_t>(B + qb, (uint8_t)v[m]);
                        gst<uint8_t>(H + qb, (uint8_t)(v[m] >> 8));
                    } else {
                        gst<uint8_t>(A + qa, (uint8_t)v[m]);
                    }
                } else {
                    gst<uint8_t>(A + qa, (uint8_t)v[m]);
                    if (big) gst<uint8_t>(H + qb, (uint8_t)(v[m] >> 8));
                }
                qa += (C3 && big) ? 0u : 1u;
                qb += big ? 1u : 0u;
            }
        }
        fa += tot & 0xFFFFu;
        fb += tot >> 16;
    }
    wave_sync();
    sizes[0] = nk;
    if (C3) {
        sizes[1] = fa;
        sizes[2] = fb;
        sizes[3] = fb;
    } else {
        sizes[1] = n;
        sizes[2] = fb;
    }
}

// C2 / C3 merge over the concatenated intermediate: keys at 0, A at keys_length, then (C3) B at
// + dA and H at + dA + dB, or (C2) H at + dA.  A read past `total` is the reference's UB -> 1.
// *consumed = one past the last H byte (decode_scalar_lh / _ll_lh return data_h).
template <bool C3>
__device__ __forceinline__ int c23_merge_wave(const uint8_t* __restrict__ in, uint64_t total, uint64_t dA, uint64_t dB,
                                              int16_t* __restrict__ out, uint32_t n, uint64_t* consumed)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint64_t nk = svb_key_length(n);
    if (n == 0) {
        *consumed = nk;
        return 0;
    }
    uint64_t pa = nk, pb = nk + dA, ph = C3 ? nk + dA + dB : nk + dA;  // running positions (wave-uniform)
    uint32_t carry = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        const uint32_t nK = full ? kSplitStep / 8 : (n - t + 7) / 8;
        if ((t >> 3) + nK > total) return 1;
        const uint32_t kb = (t >> 3) + 2u * lane;
        uint32_t kw = 0;
        if (full) {
            kw = gld<uint16_t>(in + kb);
        } else {
            if (kb < nk) kw = gb(in + kb);
            if (kb + 1 < nk) kw |= (uint32_t)gb(in + kb + 1) << 8;
        }
        const uint32_t nv = full ? 16u : lane_valid(n, t);
        kw &= nv >= 16 ? 0xFFFFu : ((1u << nv) - 1u);
        const uint32_t nb = (uint32_t)__builtin_popcount(kw), ns = nv - nb;
        const uint32_t p = ns | (nb << 16);
        const uint32_t incl = wave_incl_sum(p);
        const uint32_t tot = readlane_u32(incl, 63), ex = incl - p;
        const uint32_t ts = tot & 0xFFFFu, tb = tot >> 16;
        if (C3 ? (pa + ts > total || pb + tb > total || ph + tb > total) : (pa + ts + tb > total || ph + tb > total))
            return 1;
        uint64_t qa = C3 ? pa + (ex & 0xFFFFu) : pa + 16u * lane, qb = pb + (ex >> 16), qh = ph + (ex >> 16);
        uint32_t acc = 0, o[16];
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const bool big = (kw >> m) & 1u;
            uint32_t v = 0;
            if ((uint32_t)m < nv) {
                if (C3) {
                    v = big ? ((uint32_t)gb(in + qb) | ((uint32_t)gb(in + qh) << 8)) : (uint32_t)gb(in + qa);
                } else {
                    v = (uint32_t)gb(in + qa) | (big ? ((uint32_t)gb(in + qh) << 8) : 0u);
                }
            }
            qa += (C3 && big) ? 0u : 1u;
            qb += big ? 1u : 0u;
            qh += big ? 1u : 0u;
            acc += (uint32_t)zz_dec16((uint16_t)v);
            o[m] = acc;
        }
        if (full) store_samples16<true>(o, acc, carry, out, t, n);
        else store_samples16<false>(o, acc, carry, out, t, n);
        if (C3) {
            pa += ts;
            pb += tb;
        } else {
            pa += ts + tb;
        }
        ph += tb;
    }
    *consumed = ph;
    return 0;
}

// ---------------------------------------------------------------------------------------------
// VBZ0 split: keys (2-bit C5 classes, ceil(n/4) bytes) then the nibble stream; returns the buffer
// size.  The step's nibbles (one LDS byte each) are packed two per byte by nwin_flush.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kNibWin = 4 * kSplitStep + 64;  // carried nibbles (< 32) + 4 per sample
struct Vbz0SplitLds {
    alignas(16) uint8_t N[kNibWin];
};

__device__ __forceinline__ uint32_t nib_count(uint32_t c) { return c == 0 ? 0u : (c == 1 ? 1u : (c == 2 ? 2u : 4u)); }

__device__ __forceinline__ uint32_t vbz0_split_wave(const int16_t* __restrict__ x, uint32_t n, uint8_t* out, Vbz0SplitLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    if (n == 0) return 0;
    const uint32_t nk = (n + 3) / 4;
    uint8_t* data = out + nk;
    uint32_t fill = 0, gpos = 0, prevX = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        uint32_t v[16];
        if (full) load_deltas16<true>(x, n, t, prevX, v);
        else load_deltas16<false>(x, n, t, prevX, v);
        const uint32_t nv = full ? 16u : lane_valid(n, t);
        uint32_t kw = 0, cnt = 0;
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t c = ((uint32_t)m < nv && v[m] != 0) ? 1u + (v[m] > 16) + (v[m] > 272) : 0u;
            kw |= c << (2 * m);
            cnt += nib_count(c);
        }
        const uint32_t nK = full ? kSplitStep / 4 : (n - t + 3) / 4;
        uint8_t* kout = out + (t >> 2);
        if (4u * lane + 4u <= nK) gst<uint32_t>(kout + 4u * lane, kw);
        else for (uint32_t b = 4u * lane; b < nK; b++) gst<uint8_t>(kout + b, (uint8_t)(kw >> (8u * (b - 4u * lane))));
        const uint32_t incl = wave_incl_sum(cnt);
        uint32_t q = fill + incl - cnt;
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t c = (kw >> (2 * m)) & 3u;
            const uint32_t w = v[m] - (c == 1 ? 1u : (c == 2 ? 17u : 273u));
            const uint32_t k = nib_count(c);
            for (uint32_t j = 0; j < k; j++) W.N[q + j] = (uint8_t)((w >> (4 * j)) & 15u);
            q += k;
        }
        fill += readlane_u32(incl, 63);
        lds_sync();
        nwin_flush(W.N, fill, data, gpos);
        lds_sync();
    }
    const uint32_t nb = (fill + 1) / 2;  // a trailing odd nibble leaves its high half zero
    for (uint32_t j = lane; j < nb; j += 64) {
        const uint32_t lo = W.N[2 * j], hi = (2 * j + 1 < fill) ? W.N[2 * j + 1] : 0u;
        gst<uint8_t>(data + gpos + j, (uint8_t)(lo | (hi << 4)));
    }
    lds_sync();
    return nk + gpos + nb;
}

// VBZ0 merge over the intermediate (frame content, no padding): keys at 0, nibbles from ceil(n/4).
// *consumed = keys + ceil(nibbles / 2) (decode_scalar_VBZ1's final data pointer; 0 for n == 0).
struct Vbz0MergeLds {
    alignas(16) uint8_t D[2 * kSplitStep + 64];
};

__device__ __forceinline__ int vbz0_merge_wave(const uint8_t* __restrict__ in, uint64_t total, int16_t* __restrict__ out,
                                               uint32_t n, uint64_t* consumed, Vbz0MergeLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    if (n == 0) {
        *consumed = 0;
        return 0;
    }
    const uint64_t nk = (n + 3) / 4;
    uint64_t nib = 0;  // nibbles consumed (wave-uniform)
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
        const uint32_t nv = full ? 16u : lane_valid(n, t);
        if (nv < 16) kw &= (1u << (2u * nv)) - 1u;
        uint32_t cnt = 0;
#pragma unroll
        for (int m = 0; m < 16; m++) cnt += nib_count((kw >> (2 * m)) & 3u);
        const uint32_t incl = wave_incl_sum(cnt);
        const uint32_t tn = readlane_u32(incl, 63);
        const uint64_t b0 = nk + (nib >> 1), b1 = nk + ((nib + tn + 1) >> 1);
        if (b1 > total) return 1;
        const uint64_t w0 = stage_bytes(W.D, in, b0, (uint32_t)(b1 - b0));
        lds_sync();
        uint32_t q = (uint32_t)(2 * (nk - w0) + nib) + incl - cnt;  // window-relative nibble index
        uint32_t acc = 0, o[16];
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t c = (kw >> (2 * m)) & 3u;
            const uint32_t k = nib_count(c);
            uint32_t v = 0;
            for (uint32_t j = 0; j < k; j++) {
                const uint32_t qq = q + j;
                v |= (((uint32_t)W.D[qq >> 1] >> (4u * (qq & 1u))) & 15u) << (4 * j);
            }
            q += k;
            v = c == 0 ? 0u : v + (c == 1 ? 1u : (c == 2 ? 17u : 273u));
            acc += (uint32_t)zz_dec16((uint16_t)v);
            o[m] = acc;
        }
        if (full) store_samples16<true>(o, acc, carry, out, t, n);
        else store_samples16<false>(o, acc, carry, out, t, n);
        nib += tn;
        lds_sync();
    }
    *consumed = nk + ((nib + 1) >> 1);
    return 0;
}

}  // namespace pgn
