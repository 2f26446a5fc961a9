// pgn_vbz.h -- VBZ (svb16 + zstd) split and merge on one wave: the byte layer of the reference's
// pod5::compress_signal / decompress_signal (pod5/c++/pod5_format/signal_compression.cpp:37-78,
// 96-141), the baseline codec every input POD5 file uses.
//
// Split = svb16::encode<int16_t, /*delta*/true, /*zigzag*/true> (svb16/encode.hpp:12-24,
//         svb16/encode_scalar.hpp:18-66): keys = 1 bit per sample, LSB first, ceil(n/8) bytes
//         (svb16.h:16-20); data = 1 byte if the zig-zag delta is < 256, else 2 bytes little endian.
// Merge = svb16::decode (svb16/decode.hpp:25-37, decode_scalar.hpp:34-74) + the consumed-bytes
//         check of signal_compression.cpp:128-131.
//
// A step is 1024 samples; lane l owns the 16 consecutive samples t + 16l .. t + 16l + 15, so its 16
// key bits are one aligned 16-bit key word.  A lane's data bytes start at the step fill plus the
// byte counts of the lanes below (one DPP wave scan); bytes are written into an LDS window and
// leave as 16-byte stores (split) or are staged from HBM with 16-byte loads (merge).
#pragma once
#include "pgn_c5.h"

namespace pgn {

__host__ __device__ constexpr uint32_t svb_key_length(uint32_t n) { return (n >> 3) + (((n & 7u) + 7u) >> 3); }

struct VbzSplitLds {
    alignas(16) uint8_t D[2 * kSplitStep + 16 + 16 + 4 * 64];  // carried tail + 2 bytes per sample + discard slots
};
constexpr uint32_t kVbzDummy = 2 * kSplitStep + 32;  // + 4 * lane: per-lane discard slots

// One 1024-sample step of the split (Full: every sample exists).  Writes the step's key bytes to
// keys + t/8 and its data bytes into the window after `fill`.
template <bool Full>
__device__ __forceinline__ void vbz_split_step(const int16_t* __restrict__ x, uint32_t n, uint32_t t, uint8_t* keys, uint32_t nk,
                                               VbzSplitLds& W, uint32_t& fill, uint32_t& prevX)
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
    uint32_t v[16];
    uint32_t kw = 0, cnt = 0;
#pragma unroll
    for (int m = 0; m < 16; m++) {
        v[m] = zz_enc16((uint16_t)(xv[m] - prv));
        prv = xv[m];
        const bool valid = Full || (i0 + (uint32_t)m < n);
        kw |= (valid && v[m] > 255u) ? (1u << m) : 0u;
        cnt += valid ? 1u : 0u;
    }
    cnt += (uint32_t)__builtin_popcount(kw);
    // key word: bytes t/8 + 2l, t/8 + 2l + 1 (svb16 key bit i%8 of byte i/8)
    const uint32_t kb = (t >> 3) + 2u * lane;
    if (Full) {
        gst<uint16_t>(keys + kb, (uint16_t)kw);
    } else {
        if (kb < nk) gst<uint8_t>(keys + kb, (uint8_t)kw);
        if (kb + 1 < nk) gst<uint8_t>(keys + kb + 1, (uint8_t)(kw >> 8));
    }
    const uint32_t incl = wave_incl_sum(cnt);
    uint32_t q = fill + incl - cnt;
    const uint32_t dd = kVbzDummy + 4u * lane;
#pragma unroll
    for (int m = 0; m < 16; m++) {
        const bool valid = Full || (i0 + (uint32_t)m < n);
        const bool big = (kw >> m) & 1u;
        W.D[valid ? q : dd] = (uint8_t)v[m];
        W.D[big ? q + 1 : dd] = (uint8_t)(v[m] >> 8);
        q += (valid ? 1u : 0u) + (big ? 1u : 0u);
    }
    fill += readlane_u32(incl, 63);
}

// svb16 encode of x[0..n) into out (keys then data); returns the encoded size
// (svb16/encode.hpp:21-23: keys_length + data bytes; 0 for n == 0).
__device__ __forceinline__ uint32_t vbz_split_wave(const int16_t* __restrict__ x, uint32_t n, uint8_t* out, VbzSplitLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    if (n == 0) return 0;
    const uint32_t nk = svb_key_length(n);
    uint8_t* data = out + nk;
    uint32_t fill = 0, gpos = 0, prevX = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        if (t + kSplitStep <= n) vbz_split_step<true>(x, n, t, out, nk, W, fill, prevX);
        else vbz_split_step<false>(x, n, t, out, nk, W, fill, prevX);
        lds_sync();
        bwin_flush(W.D, fill, data, gpos);
        lds_sync();
    }
    for (uint32_t j = lane; j < fill; j += 64) gst<uint8_t>(data + gpos + j, W.D[j]);
    lds_sync();
    return nk + gpos + fill;
}

// svb16 decode of the intermediate in[0..total) into out[0..n).  Returns 0, or 1 when a key or data
// byte would be read past `total` (the reference reads past its buffer there).  *consumed = bytes
// used (keys + data; 0 for n == 0, svb16/decode_scalar.hpp:43-45).  `in` must stay readable 16
// bytes past `total` (scratch padding).
struct VbzMergeLds {
    alignas(16) uint8_t D[2 * kSplitStep + 32];
};

template <bool Full>
__device__ __forceinline__ void vbz_merge_step(const VbzMergeLds& W, uint32_t kw, uint32_t q, uint32_t& carry,
                                               int16_t* __restrict__ out, uint32_t t, uint32_t n)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t acc = 0;
    uint32_t o[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        const uint32_t big = (kw >> m) & 1u;
        const uint32_t lo = W.D[q], hi = W.D[q + 1];
        const uint32_t v = big ? (lo | (hi << 8)) : lo;
        q += 1u + big;
        acc += (uint32_t)zz_dec16((uint16_t)v);
        o[m] = acc;
    }
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

__device__ __forceinline__ int vbz_merge_wave(const uint8_t* __restrict__ in, uint64_t total, int16_t* __restrict__ out,
                                              uint32_t n, uint64_t* consumed, VbzMergeLds& W)
{
    const uint32_t lane = (uint32_t)lane_id();
    if (n == 0) {
        *consumed = 0;
        return 0;
    }
    const uint32_t nk = svb_key_length(n);
    if (nk > total) return 1;
    uint64_t dpos = nk;  // next data byte (wave-uniform)
    uint32_t carry = 0;
    for (uint32_t t = 0; t < n; t += kSplitStep) {
        const bool full = t + kSplitStep <= n;
        const uint32_t kb = (t >> 3) + 2u * lane;
        uint32_t kw = 0;
        if (full) {
            kw = gld<uint16_t>(in + kb);
        } else {
            if (kb < nk) kw = gb(in + kb);
            if (kb + 1 < nk) kw |= (uint32_t)gb(in + kb + 1) << 8;
            const uint32_t first = 16u * lane, nv = (n - t) > first ? (n - t) - first : 0u;
            if (nv < 16) kw &= (1u << nv) - 1u;
        }
        const uint32_t nv = full ? 16u : ((n - t) > 16u * lane ? ((n - t) - 16u * lane < 16u ? (n - t) - 16u * lane : 16u) : 0u);
        const uint32_t cnt = nv + (uint32_t)__builtin_popcount(kw);
        const uint32_t incl = wave_incl_sum(cnt);
        const uint32_t tot = readlane_u32(incl, 63);
        if (dpos + tot > total) return 1;
        const uint64_t w0 = stage_bytes(W.D, in, dpos, tot);
        lds_sync();
        const uint32_t q = (uint32_t)(dpos - w0) + incl - cnt;
        if (full) vbz_merge_step<true>(W, kw, q, carry, out, t, n);
        else vbz_merge_step<false>(W, kw, q, carry, out, t, n);
        dpos += tot;
        lds_sync();
    }
    *consumed = dpos;
    return 0;
}

}  // namespace pgn
