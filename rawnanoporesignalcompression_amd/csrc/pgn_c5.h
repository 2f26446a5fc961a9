// pgn_c5.h -- C5 ("N01") split and merge on one wave.
//
// Split = svb16::encode_scalar_N01<int16_t, /*delta*/true, /*zigzag*/true> (pgnano/svb16/C5.hpp:57-152)
// Merge = svb16::decode_scalar_N01 (C5.hpp:173-257) as driven by decode_N01 (C5.hpp:260-275) and
//         decompress_signal_N01's consumed-bytes check (C5.hpp:669-677).
//
// The reference walks the samples serially; here a wave takes 256 samples per step (4 per lane, one
// key byte per lane), classifies them, and places every S/M/L value with a wave prefix sum of the
// per-lane class counts.  The wrapping 16-bit delta is undone with a wave prefix sum.
#pragma once
#include "pgn_wave.h"

namespace pgn {

__device__ __forceinline__ uint16_t zz_enc16(uint16_t v) { return (uint16_t)((uint16_t)(v + v) ^ (uint16_t)((int16_t)v >> 15)); }
__device__ __forceinline__ uint16_t zz_dec16(uint16_t v) { return (uint16_t)((v >> 1) ^ (uint16_t)(0u - (v & 1u))); }

struct C5Streams {
    uint8_t *K, *S, *M, *Ll, *Lh;
};

// sizes[5] = {keys, S, M, Llow, Lhigh} bytes.  nib: >= 264 bytes of LDS.
__device__ inline void c5_split_wave(const int16_t* __restrict__ x, uint32_t n, const C5Streams& st, uint32_t sizes[5],
                                     uint8_t* nib)
{
    const int lane = lane_id();
    if (n == 0) {
        for (int i = 0; i < 5; i++) sizes[i] = 0;
        return;
    }
    uint32_t sBytes = 0, mBase = 0, lBase = 0;
    uint32_t pending = 0, pendingVal = 0;  // an unpaired S nibble carried into the next step
    uint16_t prevTile = 0;                  // last sample of the previous step
    for (uint32_t t = 0; t < n; t += 256) {
        const uint32_t i0 = t + 4u * (uint32_t)lane;
        uint16_t xs[4];
#pragma unroll
        for (int j = 0; j < 4; j++) xs[j] = (i0 + j < n) ? (uint16_t)x[i0 + j] : 0;
        uint16_t prevLane = (uint16_t)__shfl_up((int)xs[3], 1, 64);
        uint16_t prev = (lane == 0) ? prevTile : prevLane;
        unsigned code[4];
        uint16_t val[4];
        uint32_t ns = 0, nm = 0, nl = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint16_t v = zz_enc16((uint16_t)(xs[j] - prev));
            prev = xs[j];
            unsigned c = (v == 0) ? 0u : (v <= 16 ? 1u : (v <= 272 ? 2u : 3u));
            if (i0 + j >= n) c = 4;  // past the end
            code[j] = c;
            val[j] = (c == 1) ? (uint16_t)(v - 1) : (c == 2 ? (uint16_t)(v - 17) : (uint16_t)(v - 273));
            ns += (c == 1);
            nm += (c == 2);
            nl += (c == 3);
        }
        const uint32_t packed = ns | (nm << 10) | (nl << 20);
        const uint32_t incl = wave_incl_sum(packed);
        const uint32_t excl = incl - packed;
        const uint32_t tot = readlane_u32(incl, 63);
        uint32_t sR = excl & 1023, mR = (excl >> 10) & 1023, lR = (excl >> 20) & 1023;
        const uint32_t tileS = tot & 1023, tileM = (tot >> 10) & 1023, tileL = (tot >> 20) & 1023;
        if (i0 < n) {
            unsigned kb = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) kb |= (code[j] & 3u) << (2 * j);
            st.K[i0 >> 2] = (uint8_t)kb;
        }
        // S nibbles staged in LDS at [pending + rank]
        if (lane == 0 && pending) nib[0] = (uint8_t)pendingVal;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (code[j] == 1) nib[pending + sR++] = (uint8_t)val[j];
            else if (code[j] == 2) st.M[mBase + mR++] = (uint8_t)val[j];
            else if (code[j] == 3) {
                st.Ll[lBase + lR] = (uint8_t)(val[j] & 0xFF);
                st.Lh[lBase + lR] = (uint8_t)(val[j] >> 8);
                lR++;
            }
        }
        wave_sync();
        const uint32_t T = pending + tileS;
        for (uint32_t b = (uint32_t)lane; b < T / 2; b += 64)
            st.S[sBytes + b] = (uint8_t)(nib[2 * b] | (nib[2 * b + 1] << 4));
        uint32_t newPendingVal = (T & 1) ? nib[T - 1] : 0;
        wave_sync();
        sBytes += T / 2;
        pending = T & 1;
        pendingVal = newPendingVal;
        mBase += tileM;
        lBase += tileL;
        prevTile = (uint16_t)readlane_u32(xs[3], 63);
    }
    if (pending && lane == 0) st.S[sBytes] = (uint8_t)pendingVal;
    sizes[0] = (n + 3) / 4;
    sizes[1] = sBytes + pending;
    sizes[2] = mBase;
    sizes[3] = lBase;
    sizes[4] = lBase;
}

// Merge over the reference's concatenated intermediate buffer (see oracle c5_merge): stream starts at
// keys_length = ceil(n/4), then +dS, +dM, +dLl; a read past `total` is the reference's UB -> error.
// Returns 0 ok, 1 out-of-bounds; *consumed = one past the last Lhigh byte.
__device__ inline int c5_merge_wave(const uint8_t* __restrict__ in, uint64_t total, uint64_t dS, uint64_t dM,
                                    uint64_t dLl, int16_t* __restrict__ out, uint32_t n, uint64_t* consumed)
{
    const int lane = lane_id();
    const uint64_t kl = ((uint64_t)n + 3) / 4;
    const uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    uint64_t sN = 0, mN = 0, lN = 0;
    uint16_t carry = 0;
    bool bad = false;
    for (uint32_t t = 0; t < n; t += 256) {
        const uint32_t i0 = t + 4u * (uint32_t)lane;
        unsigned code[4] = {4, 4, 4, 4};
        if (i0 < n) {
            uint64_t kb = i0 >> 2;
            if (kb < total) {
                unsigned key = in[kb];
#pragma unroll
                for (int j = 0; j < 4; j++) code[j] = (i0 + j < n) ? ((key >> (2 * j)) & 3u) : 4u;
            } else {
                bad = true;
            }
        }
        uint32_t ns = 0, nm = 0, nl = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) { ns += code[j] == 1; nm += code[j] == 2; nl += code[j] == 3; }
        const uint32_t packed = ns | (nm << 10) | (nl << 20);
        const uint32_t incl = wave_incl_sum(packed);
        const uint32_t excl = incl - packed;
        const uint32_t tot = readlane_u32(incl, 63);
        uint64_t sq = sN + (excl & 1023), mq = mN + ((excl >> 10) & 1023), lq = lN + ((excl >> 20) & 1023);
        uint16_t d[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint16_t v = 0;
            if (code[j] == 1) {
                uint64_t b = ps + (sq >> 1);
                if (b < total) v = (uint16_t)(((sq & 1) ? (in[b] >> 4) : (in[b] & 15)) + 1);
                else bad = true;
                sq++;
            } else if (code[j] == 2) {
                uint64_t b = pm + mq;
                if (b < total) v = (uint16_t)(in[b] + 17);
                else bad = true;
                mq++;
            } else if (code[j] == 3) {
                uint64_t bl = pl + lq, bh = ph + lq;
                if (bl < total && bh < total) v = (uint16_t)(((unsigned)in[bh] << 8) + in[bl] + 273);
                else bad = true;
                lq++;
            }
            d[j] = (code[j] < 4) ? zz_dec16(v) : (uint16_t)0;
        }
        uint16_t s1 = (uint16_t)(d[0] + d[1]), s2 = (uint16_t)(s1 + d[2]), s3 = (uint16_t)(s2 + d[3]);
        uint32_t lincl = wave_incl_sum(s3);
        uint16_t base = (uint16_t)(carry + (uint16_t)(lincl - s3));
        uint16_t o[4] = {(uint16_t)(base + d[0]), (uint16_t)(base + s1), (uint16_t)(base + s2), (uint16_t)(base + s3)};
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (i0 + j < n) out[i0 + j] = (int16_t)o[j];
        carry = (uint16_t)(carry + (uint16_t)readlane_u32(lincl, 63));
        sN += tot & 1023;
        mN += (tot >> 10) & 1023;
        lN += (tot >> 20) & 1023;
    }
    *consumed = ph + lN;
    return ballot(bad) ? 1 : 0;
}

}  // namespace pgn
