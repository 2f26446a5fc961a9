// pgn_zdec.h -- one wave decodes the zstd frame(s) of one stream (ZSTD_decompress semantics, the
// call at C5.hpp:588-667).  Frame/block headers and the sequence list are parsed wave-uniformly;
// the Huffman table description is staged into LDS and parsed there; raw/RLE blocks, literal and
// match copies use the whole wave; the four Huffman streams of a literals section are decoded by
// all 64 lanes (16 per stream, speculative start + synchronisation, see huf_decode4_wave).
#pragma once
#include "pgn_wave.h"
#include "zstd1_dec.h"

namespace pgn {

constexpr int32_t kWinBits = 384;        // Huffman stream bits per lane per round (pgn_huf4.h)
constexpr int32_t kOvBits = 64;         // speculative overlap above a lane's window (pgn_huf4.h)
constexpr int kBmpBits = 128;            // speculative boundaries recorded per lane: bit d = position hi - d
constexpr int kStgWords = 16;            // staged bytes per lane per round: 64 >= (384 + 63) / 8 + 8

constexpr int kSeqWin = 2048;            // sequences bitstream window staged in LDS
constexpr int kSeqHdr = 400;             // staged sequences-section header (table descriptions)
constexpr int kSeqTab = 1280;            // LL [0,512) + OF [512,768) + ML [768,1280) FSE decode entries

constexpr uint32_t kJobTab = 512;     // compact table slots of a deferred job (pgn_hufjob.h; 16-bit: nbBits | symbol << 8)
constexpr uint32_t kJobTabUse = 352;  // entries a job's compact table may have: dec_huf_kernel keeps 352 per frame in LDS
constexpr unsigned kHufLdsLog = 11;  // Huffman tables up to this log live in LDS (zstd's encoders
                                     // never exceed 11); a 12-bit table is built in HBM (slow path)

// The Huffman table build's LDS (huf_build_dtable_body): part of DecLds (sDec.hb), used by the frame
// decoder and by dec_frame_fast's job-only build in dec_zstd_kernel.
struct HufBuildLds {
    uint8_t wts[256];         // weights of the current table
    uint8_t order[256];       // symbols sorted by (weight, symbol)
    uint8_t hbuf[272];        // staged Huffman table description (zero padded)
    z1::FseDEntry wdt[64];    // weights FSE decode table (tableLog <= 6)
    int16_t wnorm[16];
};

// Per-workgroup LDS, sized for four decode waves per SIMD: the literal stage (table, boundary
// bitmap, staging rows) and the sequences stage overlay each other.  A Huffman table that must
// outlive a sequences stage (treeless literals in a later block) is parked in HBM (DecScratch::htab).
struct alignas(16) DecLds {
    union {
        struct {  // literals stage
            uint16_t tab[1u << kHufLdsLog];   // Huffman decode table: symbol | nbBits << 8
            union {
                // per-lane arrays are word-major ([word][lane]): lanes touching their own rows hit distinct banks
                uint32_t stg[kStgWords][64];  // staged stream bytes of the current round
                HufBuildLds hb;               // table build only (done before the rounds start)
            };
        };
        struct {  // sequences stage
            uint32_t qtab[kSeqTab];           // FSE entries: newState | symbol << 16 | nbBits << 24
            uint32_t qsq[64][3];              // a batch of decoded sequences: litLength, matchLength, offset
            union {
                struct {                      // section head and table build (before the bitstream)
                    int16_t qnorm[64];
                    uint8_t qhdr[kSeqHdr];
                };
                uint8_t qwin[kSeqWin];        // bitstream window
            };
        };
    };
};
// 8 KiB: 20 one-wave workgroups per CU (160 KiB of LDS)
static_assert(sizeof(DecLds) <= 8192, "decoder LDS exceeds 8 KiB");

// Frame state of the sequences stage, carried across the blocks of a frame.
struct SeqState {
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;  // repeat offsets
    uint32_t valid = 0;                      // bit k: table k valid (repeat mode)
    uint32_t saved = 0;                      // bit k: table k saved to S.tables (multi-block frames)
};

// One instance per decode workgroup (namespace scope, so every access is a DS instruction).
static_assert(sizeof(DecLds) <= kCodecLdsBytes, "decoder LDS exceeds the codec LDS");
#define sDec (*reinterpret_cast<DecLds*>(sCodecLds))

struct DecScratch {
    uint8_t* lit;           // literals of a block with sequences (<= 128 KiB)
    uint32_t* seqs;         // decoded sequences: {litLength, matchLength, offset} triples
    uint32_t maxSeq;
    uint32_t* tables;       // the three sequence FSE tables of a multi-block frame (kSeqTab + 4 words)
    uint16_t* htab;         // 4096 entries: a 12-bit Huffman table, or the parked LDS table
    uint8_t* job;           // this frame's HufJob record (pgn_hufjob.h): a literals-only last block's
                            // four Huffman streams are left to dec_huf_kernel; null = decode in place
    struct CoopCmd __attribute__((address_space(3)))* coopCmd;  // cooperative decode: the section post
    __attribute__((address_space(3))) uint32_t* coopStg;         // ... and wave 0's staging rows
};

// ---------------------------------------------------------------------------------------------
// Backward bit reader over global memory (the rare single-stream case)
// ---------------------------------------------------------------------------------------------
struct RevBits {
    const uint8_t* s;
    uint64_t W;
    int32_t wlo;
};
__device__ __forceinline__ void rb_fill(RevBits& r, int32_t pos)
{
    const int32_t byteEnd = (pos + 7) >> 3;
    const int32_t byteLo = byteEnd - 8;
    if (byteLo >= 0) {
        r.W = ld64u(r.s + byteLo);
        r.wlo = byteLo * 8;
    } else {
        uint64_t v = 0;
        for (int32_t k = byteEnd - 1; k >= 0; k--) v = (v << 8) | gb(r.s + k);
        r.W = v;
        r.wlo = 0;
    }
}
__device__ __forceinline__ uint32_t rb_peek(const RevBits& r, int32_t pos, unsigned nb)
{
    const int32_t lo = pos - (int32_t)nb;
    const uint32_t m = (1u << nb) - 1;
    if (lo >= r.wlo) return (uint32_t)(r.W >> (lo - r.wlo)) & m;
    return (uint32_t)(r.W << (r.wlo - lo)) & m;  // stream start only (wlo == 0): zero bits below 0
}
// one Huffman symbol; gt = the table in HBM (12-bit tables), null = the LDS table
__device__ __forceinline__ uint32_t rb_huf(RevBits& r, int32_t& pos, unsigned tl, const uint16_t* gt)
{
    if (pos - r.wlo < (int32_t)tl && r.wlo > 0) rb_fill(r, pos);
    const uint32_t ix = rb_peek(r, pos, tl);
    const uint32_t e = gt ? (uint32_t)gld<uint16_t>(gt + ix) : (uint32_t)sDec.tab[ix];
    pos -= (int32_t)(e >> 8);
    return e & 0xFF;
}

// ---------------------------------------------------------------------------------------------
// Header window: 256 bytes of a frame held in one VGPR (lane l: bytes [base + 4l, base + 4l + 4),
// zero past the end), loaded with one coalesced access.  The frame, block and literals headers and
// the Huffman jump table are then read with v_readlane instead of a chain of dependent byte loads
// from HBM.  Bytes outside the window fall back to a global load.
// ---------------------------------------------------------------------------------------------
struct HdrWin {
    uint32_t w;
    size_t base;
};
__device__ __forceinline__ void hw_load(HdrWin& h, const uint8_t* src, size_t srcSize, size_t base)
{
    const size_t i = base + 4u * (size_t)lane_id();
    uint32_t v = 0;
    if (i + 4 <= srcSize) {
        v = ld32u(src + i);
    } else {
#pragma unroll
        for (int b = 0; b < 4; b++) v |= (i + b < srcSize) ? (uint32_t)gb(src + i + b) << (8 * b) : 0u;
    }
    h.w = v;
    h.base = base;
}
// byte at pos (wave-uniform); pos must be < the frame size the window was loaded with
__device__ __forceinline__ uint32_t hw_byte(const HdrWin& h, const uint8_t* src, size_t pos)
{
    const size_t d = pos - h.base;
    if (pos >= h.base && d < 256) return (readlane_u32(h.w, (int)(d >> 2)) >> (8 * (d & 3))) & 0xFFu;
    return gb(src + pos);
}
// little-endian 16/24/32-bit values at pos (each byte < the frame size)
__device__ __forceinline__ uint32_t hw_u16(const HdrWin& h, const uint8_t* src, size_t pos)
{
    return hw_byte(h, src, pos) | (hw_byte(h, src, pos + 1) << 8);
}
__device__ __forceinline__ uint32_t hw_u24(const HdrWin& h, const uint8_t* src, size_t pos)
{
    return hw_u16(h, src, pos) | (hw_byte(h, src, pos + 2) << 16);
}
__device__ __forceinline__ uint32_t hw_u32(const HdrWin& h, const uint8_t* src, size_t pos)
{
    return hw_u16(h, src, pos) | (hw_u16(h, src, pos + 2) << 16);
}

// ---------------------------------------------------------------------------------------------
// Four bytes of a stream of sl bytes at bytePos (any alignment); bytes outside [0, sl) read as zero.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_word(const uint8_t* s, int32_t sl, int32_t bytePos)
{
    if (bytePos >= 0 && bytePos + 4 <= sl) return ld32u(s + bytePos);
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const int32_t i = bytePos + b;
        if (i >= 0 && i < sl) v |= (uint32_t)gb(s + i) << (8 * b);
    }
    return v;
}
// Round staging: a lane's window of a round is (hi - W, hi] for an hi up to 11 bits below the
// estimate it was staged for; it stages bytes [base, base + 48) with base = 4 * floor((est - W -
// 32) / 32), so bits [q - tl, q) of every q in the window and the 64-bit reads above them are inside.
__device__ __forceinline__ int32_t round_base(int32_t hi) { return ((hi - kWinBits - 32) >> 5) * 4; }
__device__ __forceinline__ void round_load(uint4 v[kStgWords / 4], const uint8_t* s, int32_t sl, int32_t base)
{
    if (base >= 0 && base + 4 * kStgWords <= sl) {
#pragma unroll
        for (int i = 0; i < kStgWords / 4; i++) v[i] = gld<uint4>(s + base + 16 * i);
    } else {
#pragma unroll
        for (int i = 0; i < kStgWords / 4; i++)
            v[i] = make_uint4(ld_word(s, sl, base + 16 * i), ld_word(s, sl, base + 16 * i + 4),
                              ld_word(s, sl, base + 16 * i + 8), ld_word(s, sl, base + 16 * i + 12));
    }
}
// ---------------------------------------------------------------------------------------------
// Huffman table description (HUF_readStats + HUF_readDTableX1), wave-uniform over an LDS copy.
// ---------------------------------------------------------------------------------------------
// FSE_readNCount over LDS bytes already zero-padded to hb >= 8 (zstd1_dec.h fse_read_ncount).
__device__ __forceinline__ size_t ncount_lds(int16_t* norm, unsigned* maxSVPtr, unsigned* tableLogPtr, const uint8_t* istart,
                                             size_t srcSize, size_t hb, unsigned maxLogAllowed)
{
    const uint8_t* ip = istart;
    const uint8_t* iend = istart + hb;
    unsigned maxSV1 = *maxSVPtr + 1;
    int previous0 = 0;
    for (unsigned i = 0; i < maxSV1; i++) norm[i] = 0;
    uint32_t bitStream = z1::rd32(ip);
    unsigned nbBits = (bitStream & 0xF) + z1::kFseMinTableLog;
    if (nbBits > maxLogAllowed) return 0;
    bitStream >>= 4;
    int bitCount = 4;
    *tableLogPtr = nbBits;
    int remaining = (1 << nbBits) + 1;
    int threshold = 1 << nbBits;
    nbBits++;
    unsigned charnum = 0;
    while ((remaining > 1) & (charnum <= *maxSVPtr)) {
        if (previous0) {
            unsigned n0 = charnum;
            while ((bitStream & 0xFFFF) == 0xFFFF) {
                n0 += 24;
                if (ip < iend - 5) {
                    ip += 2;
                    bitStream = z1::rd32(ip) >> bitCount;
                } else {
                    bitStream >>= 16;
                    bitCount += 16;
                }
            }
            while ((bitStream & 3) == 3) {
                n0 += 3;
                bitStream >>= 2;
                bitCount += 2;
            }
            n0 += bitStream & 3;
            bitCount += 2;
            if (n0 > *maxSVPtr) return 0;
            while (charnum < n0) norm[charnum++] = 0;
            if ((ip <= iend - 7) || (ip + (bitCount >> 3) <= iend - 4)) {
                ip += bitCount >> 3;
                bitCount &= 7;
                bitStream = z1::rd32(ip) >> bitCount;
            } else {
                bitStream >>= 2;
            }
        }
        {
            int const max = (2 * threshold - 1) - remaining;
            int count;
            if ((int)(bitStream & (uint32_t)(threshold - 1)) < max) {
                count = (int)(bitStream & (uint32_t)(threshold - 1));
                bitCount += (int)nbBits - 1;
            } else {
                count = (int)(bitStream & (uint32_t)(2 * threshold - 1));
                if (count >= threshold) count -= max;
                bitCount += (int)nbBits;
            }
            count--;
            remaining -= count < 0 ? -count : count;
            norm[charnum++] = (int16_t)count;
            previous0 = !count;
            while (remaining < threshold) {
                nbBits--;
                threshold >>= 1;
            }
            if ((ip <= iend - 7) || (ip + (bitCount >> 3) <= iend - 4)) {
                ip += bitCount >> 3;
                bitCount &= 7;
            } else {
                bitCount -= (int)(8 * (iend - 4 - ip));
                ip = iend - 4;
            }
            bitStream = z1::rd32(ip) >> (bitCount & 31);
        }
    }
    if (remaining != 1) return 0;
    if (bitCount > 32) return 0;
    *maxSVPtr = charnum - 1;
    ip += (bitCount + 7) >> 3;
    const size_t used = (size_t)(ip - istart);
    if (used > srcSize) return 0;
    return used;
}

// FSE_buildDTable for the weight alphabet (tableLog <= 6, maxSV <= 12) into sDec.wdt, one table
// entry per lane.  The serial spread visits positions (k * step) & mask, skipping those above
// highThreshold (the -1 symbols' slots, assigned from the top in symbol order), and gives the k-th
// valid position to the symbol whose cumulative positive count covers k: lane u computes its
// position, its rank among the valid ones (ballot + mbcnt) and that symbol directly.  The state
// of entry u counts the earlier entries of its symbol (one ballot per symbol).
__device__ __forceinline__ bool wdtable_build(HufBuildLds& H, const int16_t* norm, unsigned maxSV, unsigned tableLog)
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t mask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    const int ns = lane <= maxSV ? norm[lane] : 0;
    const uint32_t low = ns == -1 ? 1u : 0u, cnt = ns > 0 ? (uint32_t)ns : 0u;
    const uint32_t lowIncl = wave_incl_sum(low), cntIncl = wave_incl_sum(cnt);
    const uint32_t nLow = readlane_u32(lowIncl, 63), total = readlane_u32(cntIncl, 63);
    const uint32_t highThreshold = tableSize - 1 - nLow;
    if (total != highThreshold + 1) return false;  // the serial spread's final `position != 0`
    if (low) H.wdt[tableSize - lowIncl].symbol = (uint8_t)lane;
    const uint32_t q = (lane * step) & mask;
    const bool valid = lane < tableSize && q <= highThreshold;
    const uint32_t k = mbcnt(ballot(valid));
    uint32_t sym = 0;  // number of symbols whose cumulative count is <= k
    for (unsigned sy = 0; sy <= maxSV; sy++) sym += readlane_u32(cntIncl, (int)sy) <= k ? 1u : 0u;
    if (valid) H.wdt[q].symbol = (uint8_t)sym;
    lds_sync();
    const uint32_t su = lane < tableSize ? H.wdt[lane].symbol : 0xFFu;
    uint32_t rank = 0;
    for (unsigned sy = 0; sy <= maxSV; sy++) {
        const uint64_t m = ballot(su == sy);
        rank = su == sy ? mbcnt(m) : rank;
    }
    // symbolNext starts at the normalized count (1 for a -1 symbol)
    const uint32_t start = (uint32_t)__shfl((int)(low ? 1u : cnt), (int)(su & 63u), 64);
    if (lane < tableSize) {
        const uint32_t nextState = start + rank;
        const uint32_t nb = tableLog - z1::highbit32(nextState);
        H.wdt[lane].nbBits = (uint8_t)nb;
        H.wdt[lane].newState = (uint16_t)((nextState << nb) - tableSize);
    }
    lds_sync();
    return true;
}

// Returns header bytes consumed (0 = corrupt); *tlOut = table log, *minNbOut = its shortest code.
// Fills sDec.tab, or gt (4096 entries in HBM) for a 12-bit table; JobOnly (dec_frame_fast): only the
// job's compact table, so the kernel needs no more LDS than H.
// hw: when not null, the frame's header window (loaded at frame offset 0) and src at frame offset hoff:
// the description is staged from it (lane-permute reads, no memory round trip) when it lies inside
// A deferred job's compact table (pgn_hufjob.h), three segments.  T[d] = the table entries whose code
// is longer than tl - d bits (weights <= d; rankStart[d + 1], T[0] = 0).  Entries [0, T1) stay whole,
// [T1, T2) keep one entry per 2^d1 and [T2, 2^tl) one per 2^d2 (T1 = T[d1], T2 = T[d2]); the entry of
// a peek p (the stream's next tl bits) is
//     min(p, (p >> d1) + C1, (p >> d2) + C2),  C1 = T1 - (T1 >> d1),  C2 = T1 + ((T2 - T1) >> d1) - (T2 >> d2)
// -- lines of slope 1, 2^-d1, 2^-d2 that cross at T1 and T2 (T[d] is a multiple of 2^d: the codes are
// canonical and complete).  d1 = 0 is the two-segment table of round 4.  (d1, d2) are chosen for the
// smallest table: on the bench's M / keys frames 300-345 / 190-240 entries, against 410-475 / 340-380
// with two segments.
struct JobSeg {
    uint32_t d1, d2, T1, T2, C1, C2, size;
};
__device__ __forceinline__ JobSeg job_segments(const uint32_t (&T)[8], unsigned tl)
{
    const uint32_t tsz = 1u << tl;
    JobSeg b{0, 0, 0, 0, 0, 0, tsz};
    const uint32_t dmax = tl - 1 < 7u ? tl - 1 : 7u;
#pragma unroll
    for (uint32_t d1 = 0; d1 < 7; d1++) {
#pragma unroll
        for (uint32_t d2 = d1 + 1; d2 <= 7; d2++) {
            if (d2 > dmax) continue;
            const uint32_t t1 = T[d1], t2 = T[d2];
            const uint32_t sz = t1 + ((t2 - t1) >> d1) + ((tsz - t2) >> d2);
            if (sz < b.size) {
                b.d1 = d1;
                b.d2 = d2;
                b.T1 = t1;
                b.T2 = t2;
                b.size = sz;
            }
        }
    }
    b.C1 = b.T1 - (b.T1 >> b.d1);
    b.C2 = b.T1 + ((b.T2 - b.T1) >> b.d1) - (b.T2 >> b.d2);
    return b;
}
// compact entry j -> its index in the full 2^tl-entry table
__device__ __forceinline__ uint32_t job_entry_index(const JobSeg& g, uint32_t j)
{
    return j < g.T1 ? j : (j < g.T1 + ((g.T2 - g.T1) >> g.d1) ? (j - g.C1) << g.d1 : (j - g.C2) << g.d2);
}

template <bool JobOnly = false>
__device__ __forceinline__ size_t huf_build_dtable_body(HufBuildLds& H, const uint8_t* src, size_t srcSize, unsigned* tlOut, uint16_t* gt,
                                                       unsigned* minNbOut, const HdrWin* hw = nullptr, uint32_t hoff = 0,
                                                       PhaseProf* Pp = nullptr, uint8_t* jobTab = nullptr,
                                                       uint32_t* jobKC = nullptr)
{
    const int lane = lane_id();
    src = uni(src);
    gt = uni(gt);
    srcSize = uni((uint64_t)srcSize);
    if (srcSize < 1) return 0;
    // stage the description (at most 129 bytes are part of it; the bytes read are [0, 129))
    const uint32_t nst = srcSize < 256 ? (uint32_t)srcSize : 256u;
    if (hw && hw->base == 0 && hoff + 144 <= 256) {
        for (uint32_t i = (uint32_t)lane; i < 272; i += 64) {
            const uint32_t fo = hoff + i, sl = fo >> 2 < 63 ? fo >> 2 : 63u;
            const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * sl), (int)hw->w);
            H.hbuf[i] = (i < nst && i < 144) ? (uint8_t)(v >> (8 * (fo & 3))) : (uint8_t)0;
        }
    } else {
        for (uint32_t i = (uint32_t)lane; i < 272; i += 64) H.hbuf[i] = i < nst ? gb(src + i) : (uint8_t)0;
    }
    lds_sync();
    const uint32_t iSize = H.hbuf[0];
    uint32_t nbW = 0;
    size_t used = 0;
    if (iSize >= 128) {
        nbW = iSize - 127;
        const uint32_t bytes = (nbW + 1) / 2;
        if (bytes + 1 > srcSize) return 0;
        for (uint32_t nn = 2u * (uint32_t)lane; nn < nbW; nn += 128) {
            const uint8_t v = H.hbuf[1 + nn / 2];
            H.wts[nn] = v >> 4;
            if (nn + 1 < nbW) H.wts[nn + 1] = v & 15;
        }
        used = bytes + 1;
    } else {
        if (iSize + 1 > srcSize) return 0;
        // FSE_readNCount pads a short header with zeros to 8 bytes
        if (iSize < 8 && (uint32_t)lane < 8 && (uint32_t)lane >= iSize) H.hbuf[1 + lane] = 0;
        lds_sync();
        unsigned maxSV = z1::kHufTableLogMax, tl = 0;
        const size_t nc = ncount_lds(H.wnorm, &maxSV, &tl, H.hbuf + 1, iSize, iSize < 8 ? 8 : iSize, 6);
        if (nc == 0 || nc >= iSize) return 0;
        lds_sync();
        if (!wdtable_build(H, H.wnorm, maxSV, tl)) return 0;
        // FSE weight stream: backward bit container over the staged bytes, the decode table in a
        // VGPR (entry u in lane u: newState | symbol << 16 | nbBits << 24, read with v_readlane)
        if (Pp) Pp->mark(12);
        const uint8_t* bs = H.hbuf + 1 + nc;
        const int32_t bl = (int32_t)(iSize - nc);
        const uint32_t last = bs[bl - 1];
        if (last == 0) return 0;
        int32_t pos = (bl - 1) * 8 + (int32_t)z1::highbit32(last);
        // the stream (<= 128 bytes) in one VGPR, lane l holding bytes [4l, 4l + 4) (zero past bl): a
        // refill is one readlane, and the container, the position and the states stay scalar
        uint32_t bsv = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int32_t i = 4 * lane + b;
            bsv |= (i < bl) ? ((uint32_t)bs[i] << (8 * b)) : 0u;
        }
        auto word = [&](int32_t wi) -> uint32_t {  // stream bytes [4wi, 4wi + 4), zero outside
            return (wi >= 0 && wi < 32) ? readlane_u32(bsv, wi) : 0u;
        };
        int32_t cl = ((pos >> 5) - 1) * 32;  // C holds bits [cl, cl + 64)
        uint64_t C = (uint64_t)word(cl >> 5) | ((uint64_t)word((cl >> 5) + 1) << 32);
        auto rd = [&](uint32_t nb) -> uint32_t {
            const int32_t lo = pos - (int32_t)nb;
            if (lo < cl) {
                cl -= 32;
                C = (C << 32) | word(cl >> 5);
            }
            pos = lo;
            return (uint32_t)(C >> (lo - cl)) & ((1u << nb) - 1u);
        };
        const uint32_t tsz = 1u << tl;
        const uint32_t E = ((uint32_t)lane < tsz)
                               ? (uint32_t)H.wdt[lane].newState | ((uint32_t)H.wdt[lane].symbol << 16) |
                                     ((uint32_t)H.wdt[lane].nbBits << 24)
                               : 0u;
        uint32_t st1 = rd(tl), st2 = rd(tl);
        // alternate states; stop when the stream overruns (FSE_decompress_usingDTable tail rule)
        while (true) {
            if (nbW > 253) return 0;
            const uint32_t e1 = readlane_u32(E, (int)st1);
            H.wts[nbW++] = (uint8_t)(e1 >> 16);
            st1 = (e1 & 0xFFFFu) + rd(e1 >> 24);
            if (pos < 0) { H.wts[nbW++] = (uint8_t)(readlane_u32(E, (int)st2) >> 16); break; }
            if (nbW > 253) return 0;
            const uint32_t e2 = readlane_u32(E, (int)st2);
            H.wts[nbW++] = (uint8_t)(e2 >> 16);
            st2 = (e2 & 0xFFFFu) + rd(e2 >> 24);
            if (pos < 0) { H.wts[nbW++] = (uint8_t)(readlane_u32(E, (int)st1) >> 16); break; }
        }
        used = iSize + 1;
    }
    if (Pp) Pp->mark(15);
    lds_sync();
    // HUF_readStats tail: implied last weight and table log (weights > 12 are corrupt)
    uint32_t w4[4];
    uint32_t wsum = 0, bad = 0, r1 = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t sym = 4u * (uint32_t)lane + (uint32_t)q;
        w4[q] = (sym < nbW) ? H.wts[sym] : 0u;
        bad |= w4[q] > z1::kHufTableLogMax;
        wsum += w4[q] > z1::kHufTableLogMax ? 0u : ((1u << w4[q]) >> 1);
        r1 += w4[q] == 1;
    }
    if (ballot(bad != 0)) return 0;
    const uint32_t weightTotal = wave_sum(wsum);
    if (weightTotal == 0) return 0;
    const unsigned tl = z1::highbit32(weightTotal) + 1;
    if (tl > z1::kHufTableLogMax) return 0;
    const uint32_t rest = (1u << tl) - weightTotal;
    if ((1u << z1::highbit32(rest)) != rest) return 0;
    const unsigned lastWeight = z1::highbit32(rest) + 1;
    const uint32_t rank1 = wave_sum(r1) + (lastWeight == 1);
    if ((rank1 < 2) || (rank1 & 1)) return 0;
    const unsigned nbSym = nbW + 1;
    {   // the last symbol takes the implied weight
        const uint32_t q = nbW & 3u;
        if ((uint32_t)lane == (nbW >> 2)) {
#pragma unroll
            for (int qq = 0; qq < 4; qq++) if ((uint32_t)qq == q) w4[qq] = lastWeight;
        }
        if (lane == 0) H.wts[nbW] = (uint8_t)lastWeight;
    }
    // per-weight counts and exclusive ranks of my four symbols (weights 1..12, 10 bits each)
    uint32_t rankIdx[4] = {0, 0, 0, 0};
    uint32_t cntW[13];
    uint32_t before[13];  // symbols of smaller weight, in order[] terms
    cntW[0] = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {  // weights 3g+1 .. 3g+3
        uint32_t packed = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w = w4[q];
            if (w >= 3u * g + 1 && w <= 3u * g + 3) packed += 1u << (10 * (w - 3 * g - 1));
        }
        const uint32_t incl = wave_incl_sum(packed);
        const uint32_t excl = incl - packed;
        const uint32_t tot = readlane_u32(incl, 63);
        uint32_t seen[3] = {0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w = w4[q];
            if (w >= 3u * g + 1 && w <= 3u * g + 3) {
                const uint32_t k = w - 3 * g - 1;
                rankIdx[q] = ((excl >> (10 * k)) & 1023u) + seen[k];
                seen[k]++;
            }
        }
#pragma unroll
        for (int k = 0; k < 3; k++) cntW[3 * g + 1 + k] = (tot >> (10 * k)) & 1023u;
    }
    uint32_t rankStart[13];
    {
        uint32_t nextU = 0, nextO = 0;
#pragma unroll
        for (unsigned w = 1; w <= 12; w++) {
            rankStart[w] = nextU;
            before[w] = nextO;
            if (w <= tl) nextU += cntW[w] << (w - 1);
            nextO += cntW[w];
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t sym = 4u * (uint32_t)lane + (uint32_t)q;
        if (sym < nbSym && w4[q]) H.order[before[w4[q]] + rankIdx[q]] = (uint8_t)sym;
    }
    lds_sync();
    if (JobOnly || jobTab) {
        // dec_frame_fast: the job's compact table (pgn_hufjob.h) straight from the ranks, without the
        // 2^tl-entry table.  Entries with codes longer than K = tl - d are those of weights <= d, the
        // first rankStart[d + 1] of the table; entry idx belongs to the last weight whose range starts
        // at or below it.  A table above kJobTabUse entries returns 0: the caller's general path.
        if (tl > kHufLdsLog) return 0;
        uint32_t Td[8];
#pragma unroll
        for (int d = 0; d < 8; d++) Td[d] = rankStart[d + 1];
        const JobSeg sg = job_segments(Td, tl);
        if (sg.size > kJobTabUse) return 0;
        for (uint32_t j = (uint32_t)lane; j < sg.size; j += 64) {
            const uint32_t idx = job_entry_index(sg, j);
            uint32_t w = 0, rs0 = 0, bf = 0;
#pragma unroll
            for (unsigned ww = 1; ww <= 12; ww++) {
                const bool in = ww <= tl && cntW[ww] != 0 && rankStart[ww] <= idx;
                w = in ? ww : w;
                rs0 = in ? rankStart[ww] : rs0;
                bf = in ? before[ww] : bf;
            }
            const uint32_t sym = H.order[bf + ((idx - rs0) >> (w - 1))];
            gst<uint16_t>(jobTab + 2 * j, (uint16_t)((tl + 1 - w) | (sym << 8)));
        }
        jobKC[0] = sg.d1 | (sg.d2 << 8);
        jobKC[1] = sg.C1;
        jobKC[2] = sg.C2;
        *tlOut = tl;
        uint32_t wmx = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) wmx = w4[q] > wmx ? w4[q] : wmx;
        *minNbOut = tl + 1 - wave_max(wmx);
        return used;
    }
    if constexpr (JobOnly) return 0;
    // fill weight by weight: weight w owns entries [rankStart[w], rankStart[w] + cntW[w] << (w - 1))
#pragma unroll
    for (unsigned w = 1; w <= 12; w++) {
        if (w > tl || cntW[w] == 0) continue;
        const uint32_t a = rankStart[w], end = a + (cntW[w] << (w - 1));
        const uint16_t nbb = (uint16_t)((tl + 1 - w) << 8);
        for (uint32_t u = a + (uint32_t)lane; u < end; u += 64) {
            const uint16_t e = (uint16_t)(H.order[before[w] + ((u - a) >> (w - 1))] | nbb);
            if (tl <= kHufLdsLog) sDec.tab[u] = e;
            else gst<uint16_t>(gt + u, e);
        }
    }
    lds_sync();
    uint32_t wmax = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) wmax = w4[q] > wmax ? w4[q] : wmax;
    wmax = wave_max(wmax);
    *tlOut = tl;
    *minNbOut = tl + 1 - wmax;
    return used;
}
// the frame decoder's call (one copy of the code for its many call sites); dec_frame_fast inlines the body
__device__ __noinline__ size_t huf_build_dtable_wave(const uint8_t* src, size_t srcSize, unsigned* tlOut, uint16_t* gt,
                                                     unsigned* minNbOut)
{
    return huf_build_dtable_body<false>(sDec.hb, src, srcSize, tlOut, gt, minNbOut);
}

}  // namespace pgn

#include "pgn_huf4.h"
#include "pgn_hufjob.h"

namespace pgn {

// Four streams with a 12-bit table (HBM): one lane per stream decodes serially.  zstd's own
// encoders never write such tables; this path exists for completeness of the format.
__device__ __noinline__ bool huf_decode1_lane(unsigned tl, const uint8_t* src, size_t sl, uint8_t* dst, uint32_t n,
                                              const uint16_t* gt);
__device__ __noinline__ bool huf_decode4_serial(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                                const uint16_t* gt)
{
    const int lane = lane_id();
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    if (remain < 6) return false;
    const size_t l1 = gld<uint16_t>(hp), l2 = gld<uint16_t>(hp + 2), l3 = gld<uint16_t>(hp + 4);
    if (l1 + l2 + l3 + 6 > remain) return false;
    const size_t l4 = remain - 6 - l1 - l2 - l3;
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs) return false;
    bool ok = true;
    if ((lane & 15) == 0) {
        const int k = lane >> 4;
        const size_t so = (k == 0) ? 0 : (k == 1 ? l1 : (k == 2 ? l1 + l2 : l1 + l2 + l3));
        const size_t sl = (k == 0) ? l1 : (k == 1 ? l2 : (k == 2 ? l3 : l4));
        const uint32_t nsym = (k == 3) ? rs - 3 * seg : seg;
        ok = huf_decode1_lane(tl, hp + 6 + so, sl, dst + (size_t)seg * k, nsym, gt);
    }
    return ballot(!ok) == 0;
}

// single-stream literals (< 256 symbols in zstd's encoder): lane 0
__device__ __noinline__ bool huf_decode1_lane(unsigned tl, const uint8_t* src, size_t sl, uint8_t* dst, uint32_t n,
                                              const uint16_t* gt)
{
    if (sl == 0 || gb(src + sl - 1) == 0) return false;
    int32_t pos = (int32_t)(sl - 1) * 8 + (int32_t)z1::highbit32(gb(src + sl - 1));
    RevBits rb;
    rb.s = src;
    rb_fill(rb, pos);
    for (uint32_t i = 0; i < n; i++) gst<uint8_t>(dst + i, (uint8_t)rb_huf(rb, pos, tl, gt));
    return pos == 0;
}

// ---------------------------------------------------------------------------------------------
// Sequences (ZSTD_decodeSeqHeaders + ZSTD_decodeSequence + execution), wave-uniform.  The three FSE
// decode tables are built in LDS (the predefined ones are copied from gSeqDefTab); the bitstream
// is read backwards through a window staged into LDS; sequences are decoded 64 at a time into LDS
// and executed by the whole wave.  Frame state (SeqState) is the caller's, passed by reference.
// ---------------------------------------------------------------------------------------------
__device__ uint32_t gSeqDefTab[kSeqTab + 4];  // predefined LL / OF / ML tables (+ their logs), filled once

__device__ __forceinline__ uint32_t seq_tab_off(int k) { return k == 0 ? 0u : (k == 1 ? 512u : 768u); }

// FSE_buildDTable into sDec.qtab + off, wave-uniform; symbolNext lives in a VGPR (lane s).
__device__ __forceinline__ bool qtable_build(uint32_t off, unsigned maxSV, unsigned tableLog)
{
    const int lane = lane_id();
    const int16_t* norm = sDec.qnorm;
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t mask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    uint32_t highThreshold = tableSize - 1;
    uint32_t nextV = 0;
    for (unsigned sy = 0; sy <= maxSV; sy++) {
        const int nv = norm[sy];
        if (nv == -1) sDec.qtab[off + highThreshold--] = sy << 16;
        nextV = (lane == (int)sy) ? (uint32_t)(nv == -1 ? 1 : nv) : nextV;
    }
    uint32_t position = 0;
    for (unsigned sy = 0; sy <= maxSV; sy++) {
        const int nv = norm[sy];
        for (int i = 0; i < nv; i++) {
            sDec.qtab[off + position] = sy << 16;
            position = (position + step) & mask;
            while (position > highThreshold) position = (position + step) & mask;
        }
    }
    if (position != 0) return false;
    lds_sync();
    for (uint32_t u = 0; u < tableSize; u++) {
        const uint32_t sy = (sDec.qtab[off + u] >> 16) & 0xFFu;
        const uint32_t nextState = readlane_u32(nextV, (int)sy);
        nextV = (lane == (int)sy) ? nextState + 1 : nextV;
        const uint32_t nb = tableLog - z1::highbit32(nextState);
        sDec.qtab[off + u] = ((nextState << nb) - tableSize) | (sy << 16) | (nb << 24);
    }
    lds_sync();
    return true;
}

// one-time build of the predefined tables (launched once per context, one wave)
__global__ __launch_bounds__(64) void seq_default_tables_kernel()
{
    const int lane = lane_id();
#pragma unroll 1
    for (int k = 0; k < 3; k++) {
        const unsigned dmax = k == 0 ? z1::kMaxLL : (k == 1 ? z1::kDefaultMaxOff : z1::kMaxML);
        const unsigned lg = k == 0 ? z1::kLLDefaultNormLog : (k == 1 ? z1::kOFDefaultNormLog : z1::kMLDefaultNormLog);
        if ((unsigned)lane <= dmax)
            sDec.qnorm[lane] = k == 0 ? z1::ll_default_norm(lane) : (k == 1 ? z1::of_default_norm(lane) : z1::ml_default_norm(lane));
        lds_sync();
        qtable_build(seq_tab_off(k), dmax, lg);
        for (uint32_t u = (uint32_t)lane; u < (1u << lg); u += 64) gSeqDefTab[seq_tab_off(k) + u] = sDec.qtab[seq_tab_off(k) + u];
        if (lane == 0) gSeqDefTab[kSeqTab + k] = lg;
        lds_sync();
    }
}

// backward bit reader over the sequences bitstream [0, len) of `bs` (global), through an LDS window
struct SeqBits {
    const uint8_t* bs;
    int32_t len;
    int32_t pos;   // unread bits
    int32_t wb;    // first stream byte held in sDec.qwin
    uint64_t C;    // stream bits [cl, cl + 64)
    int32_t cl;
};
__device__ __forceinline__ void seqbits_stage(SeqBits& b, int32_t needByte)
{
    // window [wb, wb + kSeqWin) ending just above the byte needed (or the stream end)
    int32_t top = needByte + 16 < b.len ? needByte + 16 : b.len;
    int32_t wb = top - kSeqWin;
    wb = wb < 0 ? 0 : wb;
    const int lane = lane_id();
    for (int32_t i = lane * 16; i < kSeqWin; i += 64 * 16) {
        const int32_t g = wb + i;
        if (g + 16 <= b.len) {
            *(uint4*)(sDec.qwin + i) = gld<uint4>(b.bs + g);
        } else {
            for (int t = 0; t < 16; t++) sDec.qwin[i + t] = (g + t < b.len) ? gb(b.bs + g + t) : (uint8_t)0;
        }
    }
    b.wb = wb;
    lds_sync();
}
__device__ __forceinline__ uint32_t seqbits_word(SeqBits& b, int32_t wi)  // stream bytes [4wi, 4wi + 4)
{
    const int32_t g = 4 * wi;
    if (g + 4 <= 0 || g >= b.len) return 0u;
    if (g < b.wb || g + 4 > b.wb + kSeqWin) seqbits_stage(b, g + 3 > 0 ? g + 3 : 0);
    uint32_t v = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int32_t i = g + t;
        v |= (i >= 0 && i < b.len) ? ((uint32_t)sDec.qwin[i - b.wb] << (8 * t)) : 0u;
    }
    return v;
}
__device__ __forceinline__ uint32_t seqbits_read(SeqBits& b, uint32_t nb)
{
    if (nb == 0) return 0;
    const int32_t lo = b.pos - (int32_t)nb;
    if (lo < b.cl) {
        b.cl -= 32;
        b.C = (b.C << 32) | seqbits_word(b, b.cl >> 5);
    }
    b.pos = lo;
    return (uint32_t)(b.C >> (lo - b.cl)) & (uint32_t)((1ull << nb) - 1ull);
}

// The execution of a frame's first block when all its sequences (nb <= 64, decoded into sDec.qsq) are
// one batch (on the C5 data the Lhigh frame: ~18 sequences, ~1.2 KB): the checks exec_sequences_wave's
// loop makes per sequence, for all of them at once (the first failing sequence's first failing check
// wins, as in the loop; then a bitstream not consumed to its first bit, brBad; then the trailing
// literals' room).  A block that fits runs in LDS -- literals staged into the freed bitstream window,
// the output built in the freed FSE tables, matches copied LDS to LDS, one store pass at the end --
// instead of a global-memory round trip per literal run and per match; a larger one runs the loop's
// global-memory copies.  A call in tail position, so the caller keeps nothing live across it (its
// registers bound the decode kernels' occupancy).  Returns the new output position or a DecErr.
__device__ __noinline__ long exec_one_batch(const uint8_t* lit, size_t rs, uint8_t* dst, size_t op, size_t dstCap,
                                            uint32_t nb, bool brBad)
{
    const int lane = lane_id();
    lit = uni(lit);
    rs = uni((uint64_t)rs);
    dst = uni(dst);
    op = uni((uint64_t)op);
    dstCap = uni((uint64_t)dstCap);
    nb = uni(nb);
    {
        const bool in = (uint32_t)lane < nb;
        const uint32_t sll = in ? sDec.qsq[lane][0] : 0u, sml = in ? sDec.qsq[lane][1] : 0u;
        const uint32_t sof = in ? sDec.qsq[lane][2] : 0u;
        const uint32_t llIncl = wave_incl_sum(sll), outIncl = wave_incl_sum(sll + sml);
        const uint32_t o0 = outIncl - sll - sml;      // this sequence's output offset in the block
        const bool e1 = in && (size_t)llIncl > rs;    // literals beyond the section
        const bool e2 = in && op + outIncl > dstCap;  // output beyond the destination
        const bool e3 = in && sof > o0 + sll;         // match before the frame start
        const uint64_t em = ballot(e1 || e2 || e3);
        if (em) {
            const int ft = (int)__builtin_ctzll(em);
            return readlane_u32(e1 ? 1u : (e2 ? 2u : 3u), ft) == 2u ? (long)z1::kDecErrDstSmall : (long)z1::kDecErrCorrupt;
        }
        if (brBad) return z1::kDecErrCorrupt;
        const size_t remLit = rs - readlane_u32(llIncl, 63);
        const uint32_t totOut = readlane_u32(outIncl, 63);
        if (op + totOut + remLit > dstCap) return z1::kDecErrDstSmall;
        constexpr uint32_t kOut = 4096;  // output bytes held in sDec.qtab (5,120 B)
        if ((size_t)totOut + remLit > kOut || rs > (size_t)kSeqWin) {  // too large for LDS: global copies
            size_t o = op, litPos = 0;
            for (uint32_t t = 0; t < nb; t++) {
                const uint32_t ll = sDec.qsq[t][0], ml = sDec.qsq[t][1], off = sDec.qsq[t][2];
                wave_copy(dst + o, lit + litPos, ll);
                litPos += ll;
                o += ll;
                lds_sync();
                if (off >= 64 || off >= ml) {
                    for (uint32_t k = (uint32_t)lane; k < ml; k += 64) gst<uint8_t>(dst + o + k, gb(dst + o - off + k));
                } else {
                    uint32_t r = (uint32_t)lane % off;
                    const uint32_t adv = 64u % off;
                    for (uint32_t k = (uint32_t)lane; k < ml; k += 64) {
                        gst<uint8_t>(dst + o + k, gb(dst + o - off + r));
                        r += adv;
                        r = r >= off ? r - off : r;
                    }
                }
                o += ml;
                lds_sync();
            }
            wave_copy(dst + o, lit + litPos, rs - litPos);
            o += rs - litPos;
            lds_sync();
            return (long)o;
        }
    }
    uint8_t* const ob = (uint8_t*)sDec.qtab;
    uint8_t* const lb = sDec.qwin;
    const uint32_t n = (uint32_t)rs;
    for (uint32_t i = (uint32_t)lane * 16; i < n; i += 1024) {
        if (i + 16 <= n) {
            *(uint4*)(lb + i) = gld<uint4>(lit + i);
        } else {
            for (uint32_t k = i; k < n; k++) lb[k] = gb(lit + k);
        }
    }
    lds_sync();
    uint32_t o = 0, lp = 0;
    for (uint32_t t = 0; t < nb; t++) {
        const uint32_t ll = sDec.qsq[t][0], ml = sDec.qsq[t][1], off = sDec.qsq[t][2];
        for (uint32_t k = (uint32_t)lane; k < ll; k += 64) ob[o + k] = lb[lp + k];
        o += ll;
        lp += ll;
        lds_sync();
        if (off >= 64 || off >= ml) {  // no overlap within a 64-byte step
            for (uint32_t k = (uint32_t)lane; k < ml; k += 64) {
                ob[o + k] = ob[o - off + k];
                lds_sync();
            }
        } else {  // repeating pattern of period off
            uint32_t r = (uint32_t)lane % off;
            const uint32_t adv = 64u % off;
            for (uint32_t k = (uint32_t)lane; k < ml; k += 64) {
                ob[o + k] = ob[o - off + r];
                r += adv;
                r = r >= off ? r - off : r;
                lds_sync();
            }
        }
        o += ml;
        lds_sync();
    }
    for (uint32_t k = (uint32_t)lane; k < n - lp; k += 64) ob[o + k] = lb[lp + k];
    o += n - lp;
    lds_sync();
    for (uint32_t i = (uint32_t)lane; i < o; i += 64) gst<uint8_t>(dst + op + i, ob[i]);
    lds_sync();
    return (long)(op + o);
}

// One block's sequences: decode + execute.  Returns the new output position or a negative DecErr.
__device__ __noinline__ long exec_sequences_wave(const uint8_t* seqSrc, size_t seqSize, const uint8_t* lit, size_t rs,
                                                 uint8_t* dst, size_t op, size_t dstCap, size_t frameStart,
                                                 DecScratch S, bool lastBlock, SeqState& fs, PhaseProf& P)
{
    const int lane = lane_id();
    seqSrc = uni(seqSrc);
    seqSize = uni((uint64_t)seqSize);
    lit = uni(lit);
    rs = uni((uint64_t)rs);
    dst = uni(dst);
    op = uni((uint64_t)op);
    dstCap = uni((uint64_t)dstCap);
    frameStart = uni((uint64_t)frameStart);
    S.seqs = uni(S.seqs);
    S.maxSeq = uni(S.maxSeq);
    S.tables = uni(S.tables);
    // stage the section head (nbSeq, modes, table descriptions), zero padded
    const uint32_t nst = seqSize < (size_t)kSeqHdr - 16 ? (uint32_t)seqSize : (uint32_t)kSeqHdr - 16;
    for (uint32_t i = (uint32_t)lane; i < (uint32_t)kSeqHdr; i += 64) sDec.qhdr[i] = i < nst ? gb(seqSrc + i) : (uint8_t)0;
    lds_sync();
    const int32_t srcSize = (int32_t)seqSize;
    uint32_t nbSeq = sDec.qhdr[0];
    int32_t pos = 1;
    if (nbSeq >= 128) {
        if (nbSeq == 255) {
            if (srcSize < 3) return z1::kDecErrCorrupt;
            nbSeq = ((uint32_t)sDec.qhdr[1] | ((uint32_t)sDec.qhdr[2] << 8)) + 0x7F00;
            pos = 3;
        } else {
            if (srcSize < 2) return z1::kDecErrCorrupt;
            nbSeq = ((nbSeq - 128) << 8) + sDec.qhdr[1];
            pos = 2;
        }
    }
    uint32_t rep0 = uni(fs.rep0), rep1 = uni(fs.rep1), rep2 = uni(fs.rep2);
    uint32_t valid = uni(fs.valid);
    const uint32_t saved = uni(fs.saved);
    if (nbSeq == 0) {
        if (pos != srcSize) return z1::kDecErrCorrupt;
    } else {
        if (nbSeq > S.maxSeq || pos >= srcSize) return z1::kDecErrCorrupt;
        const uint32_t modes = sDec.qhdr[pos++];
        uint32_t tlog[3];
#pragma unroll 1
        for (int k = 0; k < 3; k++) {
            const unsigned mode = (modes >> (6 - 2 * k)) & 3u;
            const uint32_t off = seq_tab_off(k);
            const unsigned maxS = k == 0 ? z1::kMaxLL : (k == 1 ? z1::kMaxOff : z1::kMaxML);
            const unsigned maxLog = k == 0 ? z1::kLLFSELog : (k == 1 ? z1::kOffFSELog : z1::kMLFSELog);
            if (mode == z1::kSetBasic) {
                const uint32_t lg = gSeqDefTab[kSeqTab + k];
                for (uint32_t u = (uint32_t)lane; u < (1u << lg); u += 64) sDec.qtab[off + u] = gSeqDefTab[off + u];
                tlog[k] = lg;
            } else if (mode == z1::kSetRle) {
                if (pos >= srcSize || sDec.qhdr[pos] > maxS) return z1::kDecErrCorrupt;
                if (lane == 0) sDec.qtab[off] = (uint32_t)sDec.qhdr[pos] << 16;
                tlog[k] = 0;
                pos += 1;
            } else if (mode == z1::kSetCompressed) {
                if (pos >= kSeqHdr - 16) return z1::kDecErrCorrupt;  // description beyond the staged head
                unsigned maxSV = maxS, tl = 0;
                const int32_t avail = srcSize - pos;
                const size_t nc = ncount_lds(sDec.qnorm, &maxSV, &tl, sDec.qhdr + pos, (size_t)avail,
                                             avail < 8 ? 8 : (size_t)avail, maxLog);
                if (nc == 0) return z1::kDecErrCorrupt;
                lds_sync();
                if (!qtable_build(off, maxSV, tl)) return z1::kDecErrCorrupt;
                tlog[k] = tl;
                pos += (int32_t)nc;
            } else {  // repeat: the previous block's table (saved to HBM)
                if (!((valid >> k) & 1u) || !((saved >> k) & 1u)) return z1::kDecErrCorrupt;
                const uint32_t lg = S.tables[kSeqTab + k];
                for (uint32_t u = (uint32_t)lane; u < (1u << lg); u += 64) sDec.qtab[off + u] = S.tables[off + u];
                tlog[k] = lg;
            }
            valid |= 1u << k;
            lds_sync();
        }
        if (!lastBlock) {  // a later block may repeat these tables
            for (int k = 0; k < 3; k++) {
                const uint32_t off = seq_tab_off(k);
                for (uint32_t u = (uint32_t)lane; u < (1u << tlog[k]); u += 64) gst<uint32_t>(S.tables + off + u, sDec.qtab[off + u]);
                if (lane == 0) gst<uint32_t>(S.tables + kSeqTab + k, tlog[k]);
            }
            fs.saved = 7u;
        }
        P.mark(9);
        // bitstream
        SeqBits br;
        br.bs = seqSrc + pos;
        br.len = srcSize - pos;
        if (br.len <= 0) return z1::kDecErrCorrupt;
        const uint8_t lastB = gb(br.bs + br.len - 1);
        if (lastB == 0) return z1::kDecErrCorrupt;
        br.pos = (br.len - 1) * 8 + (int32_t)z1::highbit32(lastB);
        seqbits_stage(br, br.len - 1);
        br.cl = ((br.pos >> 5) - 1) * 32;
        br.C = (uint64_t)seqbits_word(br, br.cl >> 5) | ((uint64_t)seqbits_word(br, (br.cl >> 5) + 1) << 32);
        uint32_t sLL = seqbits_read(br, tlog[0]);
        uint32_t sOF = seqbits_read(br, tlog[1]);
        uint32_t sML = seqbits_read(br, tlog[2]);
        size_t litPos = 0;
        P.mark(10);
        for (uint32_t b0 = 0; b0 < nbSeq; b0 += 64) {
            const uint32_t nb = (nbSeq - b0) < 64u ? nbSeq - b0 : 64u;
            // decode a batch
            for (uint32_t t = 0; t < nb; t++) {
                const uint32_t eLL = sDec.qtab[sLL], eOF = sDec.qtab[512 + sOF], eML = sDec.qtab[768 + sML];
                const uint32_t ofCode = (eOF >> 16) & 0xFFu, mlCode = (eML >> 16) & 0xFFu, llCode = (eLL >> 16) & 0xFFu;
                if (ofCode > 31) return z1::kDecErrCorrupt;
                const uint32_t ofv = (1u << ofCode) + seqbits_read(br, ofCode);
                const uint32_t mlen = z1::ml_base(mlCode) + seqbits_read(br, z1::ml_bits(mlCode));
                const uint32_t llen = z1::ll_base(llCode) + seqbits_read(br, z1::ll_bits(llCode));
                uint32_t offset;
                if (ofv > 3) {
                    offset = ofv - 3;
                    rep2 = rep1;
                    rep1 = rep0;
                    rep0 = offset;
                } else {
                    const unsigned idx = ofv - 1 + (llen == 0 ? 1u : 0u);
                    if (idx == 0) {
                        offset = rep0;
                    } else {
                        offset = (idx == 3) ? rep0 - 1 : (idx == 1 ? rep1 : rep2);
                        if (offset == 0) offset = 1;
                        if (idx != 1) rep2 = rep1;
                        rep1 = rep0;
                        rep0 = offset;
                    }
                }
                if (b0 + t + 1 < nbSeq) {
                    sLL = (eLL & 0xFFFFu) + seqbits_read(br, eLL >> 24);
                    sML = (eML & 0xFFFFu) + seqbits_read(br, eML >> 24);
                    sOF = (eOF & 0xFFFFu) + seqbits_read(br, eOF >> 24);
                }
                if (lane == 0) {
                    sDec.qsq[t][0] = llen;
                    sDec.qsq[t][1] = mlen;
                    sDec.qsq[t][2] = offset;
                }
            }
            lds_sync();
            P.mark(13);
#ifndef PGN_SEQ_LDS_OFF
            if (nbSeq <= 64 && op == frameStart) {  // a frame's first block, one batch: the rest is exec_one_batch's
                fs.rep0 = rep0;
                fs.rep1 = rep1;
                fs.rep2 = rep2;
                fs.valid = valid;
                const long r = exec_one_batch(lit, rs, dst, op, dstCap, nb, br.pos != 0);
                P.mark(15);
                return r;
            }
#endif
            // execute the batch
            for (uint32_t t = 0; t < nb; t++) {
                const uint32_t ll = sDec.qsq[t][0], ml = sDec.qsq[t][1], off = sDec.qsq[t][2];
                if (litPos + ll > rs) return z1::kDecErrCorrupt;
                if (op + ll + ml > dstCap) return z1::kDecErrDstSmall;
                wave_copy(dst + op, lit + litPos, ll);
                litPos += ll;
                op += ll;
                if ((size_t)off > op - frameStart) return z1::kDecErrCorrupt;
                lds_sync();
                if (off >= 64 || off >= ml) {  // no overlap within a 64-byte step
                    for (uint32_t k = (uint32_t)lane; k < ml; k += 64) gst<uint8_t>(dst + op + k, gb(dst + op - off + k));
                } else {  // repeating pattern of period off: byte k = pattern[k mod off]
                    uint32_t r = (uint32_t)lane % off;
                    const uint32_t adv = 64u % off;
                    for (uint32_t k = (uint32_t)lane; k < ml; k += 64) {
                        gst<uint8_t>(dst + op + k, gb(dst + op - off + r));
                        r += adv;
                        r = r >= off ? r - off : r;
                    }
                }
                op += ml;
                lds_sync();
            }
            P.mark(14);
        }
        if (br.pos != 0) return z1::kDecErrCorrupt;
        const size_t remLit = rs - litPos;
        if (op + remLit > dstCap) return z1::kDecErrDstSmall;
        wave_copy(dst + op, lit + litPos, remLit);
        op += remLit;
        lds_sync();
        P.mark(15);
        fs.rep0 = rep0;
        fs.rep1 = rep1;
        fs.rep2 = rep2;
        fs.valid = valid;
        return (long)op;
    }
    // no sequences: the literals are the block
    if (op + rs > dstCap) return z1::kDecErrDstSmall;
    wave_copy(dst + op, lit, rs);
    op += rs;
    lds_sync();
    return (long)op;
}

// Cooperative decode (small batches, dec_zstd_coop_kernel): a workgroup of kCoopWaves waves per
// frame.  Wave 0 runs zstd_decompress_wave<true>; at a four-stream Huffman section it posts the
// section here and the four waves decode one stream each with 64 lanes (huf_decode1of4_wave64);
// everything else is wave 0's.  The other waves wait in coop_helper_wave.
struct CoopCmd {
    const uint8_t* hp;
    uint8_t* dst;
    uint64_t remain;
    uint32_t rs, jt01, jt2, tl;
    uint32_t done;  // no more sections: the helpers leave
    uint32_t bad;   // a helper's stream failed
};
typedef __attribute__((address_space(3))) CoopCmd lds_cmd;

__device__ __noinline__ void coop_helper_wave(int wid, lds_cmd* cmd, lds_u32* stg, PhaseProf& P)
{
    while (true) {
        __syncthreads();  // B1: a section (or done) is posted
        if (cmd->done) break;
        const bool ok = huf_decode1of4_wave64(cmd->tl, cmd->hp, cmd->remain, cmd->dst, cmd->rs, cmd->jt01, cmd->jt2,
                                              wid, stg, P);
        if (!ok && lane_id() == 0) cmd->bad = 1;
        __syncthreads();  // B2: every stream of the section is decoded
    }
}
// wave 0's side of one section
__device__ __forceinline__ bool coop_section(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                             uint32_t jt01, uint32_t jt2, lds_cmd* cmd, lds_u32* stg, PhaseProf& P)
{
    if (lane_id() == 0) {
        cmd->hp = hp;
        cmd->dst = dst;
        cmd->remain = remain;
        cmd->rs = rs;
        cmd->jt01 = jt01;
        cmd->jt2 = jt2;
        cmd->tl = tl;
        cmd->done = 0;
        cmd->bad = 0;
    }
    __syncthreads();  // B1
    const bool ok = huf_decode1of4_wave64(tl, hp, remain, dst, rs, jt01, jt2, 0, stg, P);
    __syncthreads();  // B2
    return ok && cmd->bad == 0;
}
// wave 0 releases the helpers after its frame
__device__ __forceinline__ void coop_finish(lds_cmd* cmd)
{
    if (lane_id() == 0) cmd->done = 1;
    __syncthreads();  // B1 with done set
}

// ZSTD_decompress(dst, dstCap, src, srcSize).  Returns size or a negative z1::DecErr.  COOP: wave 0
// of a dec_zstd_coop_kernel workgroup (four-stream Huffman sections shared with the other waves).
template <bool COOP = false>
__device__ __noinline__ long zstd_decompress_wave(const uint8_t* __restrict__ src, size_t srcSize, uint8_t* __restrict__ dst,
                                                  size_t dstCap, DecScratch S, PhaseProf& P)
{
    const int lane = lane_id();
    src = uni(src);
    srcSize = uni((uint64_t)srcSize);
    dst = uni(dst);
    dstCap = uni((uint64_t)dstCap);
    S.lit = uni(S.lit);
    S.seqs = uni(S.seqs);
    S.maxSeq = uni(S.maxSeq);
    S.tables = uni(S.tables);
    S.htab = uni(S.htab);
    S.job = uni(S.job);
    P.mark(3);  // the work unit's fetch (queue, unit record) up to here
    size_t ip = 0, op = 0;
    if (srcSize == 0) return z1::kDecErrSrcSmall;
    HdrWin hw;
    while (ip < srcSize) {
        if (srcSize - ip < 4) return z1::kDecErrSrcSmall;
        hw_load(hw, src, srcSize, ip);
        const uint32_t magic = hw_u32(hw, src, ip);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (srcSize - ip < 8) return z1::kDecErrSrcSmall;
            uint32_t fs = hw_u32(hw, src, ip + 4);
            if (fs > srcSize - ip - 8) return z1::kDecErrSrcSmall;
            ip += 8 + (size_t)fs;
            continue;
        }
        if (magic != z1::kMagic) return z1::kDecErrHeader;
        if (srcSize - ip < 6) return z1::kDecErrSrcSmall;
        const uint8_t fhd = (uint8_t)hw_byte(hw, src, ip + 4);
        const unsigned dictIDFlag = fhd & 3, checksum = (fhd >> 2) & 1, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
        if (fhd & 0x08) return z1::kDecErrHeader;
        size_t hpos = ip + 5 + (singleSegment ? 0 : 1);
        const unsigned didSize = dictIDFlag == 0 ? 0 : (dictIDFlag == 1 ? 1 : (dictIDFlag == 2 ? 2 : 4));
        if (hpos + didSize > srcSize) return z1::kDecErrSrcSmall;
        uint32_t dictID = 0;
        for (unsigned k = 0; k < didSize; k++) dictID |= hw_byte(hw, src, hpos + k) << (8 * k);
        hpos += didSize;
        if (dictID != 0) return z1::kDecErrHeader;
        const unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
        if (hpos + fcsSize > srcSize) return z1::kDecErrSrcSmall;
        uint64_t fcs = 0;
        if (fcsSize == 1) fcs = hw_byte(hw, src, hpos);
        else if (fcsSize == 2) fcs = (uint64_t)hw_u16(hw, src, hpos) + 256;
        else if (fcsSize == 4) fcs = hw_u32(hw, src, hpos);
        else if (fcsSize == 8) fcs = (uint64_t)hw_u32(hw, src, hpos) | ((uint64_t)hw_u32(hw, src, hpos + 4) << 32);
        hpos += fcsSize;
        ip = hpos;
        const size_t frameStart = op;
        P.count(13);
        bool hufValid = false;  // a Huffman table exists for treeless literals
        bool hufInLds = false;  // ... and is in sDec.tab (tables up to kHufLdsLog)
        bool hufParked = false; // ... and a copy is parked in S.htab
        unsigned hufTl = 0;
        SeqState fs;  // frame state of the sequences stage: repeat offsets, table validity
        while (true) {
            if (srcSize - ip < 3) return z1::kDecErrSrcSmall;
            if (ip - hw.base + 8 > 256) hw_load(hw, src, srcSize, ip);  // a later block: headers at its start
            const uint32_t bh = hw_u24(hw, src, ip);
            ip += 3;
            const unsigned last = bh & 1, btype = (bh >> 1) & 3;
            P.count(12);
            const size_t bsize = bh >> 3;
            if (btype == 3) return z1::kDecErrCorrupt;
            if (btype == z1::kBtRaw) {
                if (bsize > srcSize - ip) return z1::kDecErrSrcSmall;
                if (op + bsize > dstCap) return z1::kDecErrDstSmall;
                wave_copy8(dst + op, src + ip, bsize);
                P.count(14, bsize);
                ip += bsize;
                op += bsize;
                P.mark(5);
            } else if (btype == z1::kBtRle) {
                if (ip + 1 > srcSize) return z1::kDecErrSrcSmall;
                if (op + bsize > dstCap) return z1::kDecErrDstSmall;
                wave_fill(dst + op, (uint8_t)hw_byte(hw, src, ip), bsize);
                ip += 1;
                op += bsize;
            } else {
                if (bsize > srcSize - ip) return z1::kDecErrSrcSmall;
                if (bsize > z1::kMaxSrc) return z1::kDecErrCorrupt;
                const uint8_t* blk = src + ip;
                // ---- literals section header
                if (bsize < 1) return z1::kDecErrCorrupt;
                const uint32_t b0 = hw_byte(hw, src, ip);
                const unsigned ltype = b0 & 3, sf = (b0 >> 2) & 3;
                size_t lh, rs, cs = 0;
                bool single = false;
                if (ltype == z1::kSetBasic || ltype == z1::kSetRle) {
                    if (sf == 0 || sf == 2) { lh = 1; rs = b0 >> 3; }
                    else if (sf == 1) { if (bsize < 2) return z1::kDecErrCorrupt; lh = 2; rs = (b0 >> 4) + ((size_t)hw_byte(hw, src, ip + 1) << 4); }
                    else { if (bsize < 3) return z1::kDecErrCorrupt; lh = 3; rs = (b0 >> 4) + ((size_t)hw_byte(hw, src, ip + 1) << 4) + ((size_t)hw_byte(hw, src, ip + 2) << 12); }
                    cs = (ltype == z1::kSetBasic) ? rs : 1;
                } else {
                    if (bsize < 5) return z1::kDecErrCorrupt;
                    const uint32_t lhc = hw_u32(hw, src, ip);
                    if (sf <= 1) { lh = 3; single = (sf == 0); rs = (lhc >> 4) & 0x3FF; cs = (lhc >> 14) & 0x3FF; }
                    else if (sf == 2) { lh = 4; rs = (lhc >> 4) & 0x3FFF; cs = lhc >> 18; }
                    else { lh = 5; rs = (lhc >> 4) & 0x3FFFF; cs = (lhc >> 22) + ((size_t)hw_byte(hw, src, ip + 4) << 10); }
                }
                if (rs > z1::kMaxSrc || lh + cs > bsize) return z1::kDecErrCorrupt;
                const uint8_t* seqSrc = blk + lh + cs;
                const size_t seqSize = bsize - lh - cs;
                if (seqSize < 1) return z1::kDecErrCorrupt;
                const bool noSeq = (hw_byte(hw, src, ip + lh + cs) == 0);
                if (noSeq && seqSize != 1) return z1::kDecErrCorrupt;
                if (noSeq && op + rs > dstCap) return z1::kDecErrDstSmall;
                uint8_t* litOut = noSeq ? dst + op : S.lit;
                const uint8_t* lit = litOut;
                P.mark(7);
                if (ltype == z1::kSetBasic) {
                    if (noSeq) wave_copy(litOut, blk + lh, rs);
                    else lit = blk + lh;
                    P.mark(5);
                } else if (ltype == z1::kSetRle) {
                    wave_fill(litOut, (uint8_t)hw_byte(hw, src, ip + lh), rs);
                    P.mark(5);
                } else {
                    const uint8_t* hp = blk + lh;
                    size_t remain = cs;
                    if (ltype == z1::kSetCompressed) {
                        unsigned tlNew = 0, mnNew = 1;
                        const size_t hsz = huf_build_dtable_wave(hp, remain, &tlNew, S.htab, &mnNew);
                        P.count(9);
                        P.mark(1);
                        if (hsz == 0) return z1::kDecErrHufTable;
                        hufValid = true;
                        hufTl = tlNew;
                        hufInLds = tlNew <= kHufLdsLog;
                        hufParked = !hufInLds;
                        hp += hsz;
                        remain -= hsz;
                    } else if (!hufValid) {
                        return z1::kDecErrCorrupt;
                    } else if (!hufInLds && hufTl <= kHufLdsLog) {  // bring the parked table back
                        for (uint32_t i = (uint32_t)lane; i < (1u << hufTl); i += 64) sDec.tab[i] = gld<uint16_t>(S.htab + i);
                        hufInLds = true;
                        lds_sync();
                    }
                    const uint16_t* gt = (hufTl <= kHufLdsLog) ? nullptr : S.htab;
                    bool ok = true;
                    if (single) {
                        if (lane == 0) ok = huf_decode1_lane(hufTl, hp, remain, litOut, (uint32_t)rs, gt);
                    } else if (gt) {
                        ok = huf_decode4_serial(hufTl, hp, remain, litOut, (uint32_t)rs, gt);
                    } else {
                        if (remain < 6) {
                            ok = false;
                        } else {
                            const size_t jp = (size_t)(hp - src);  // the jump table, from the header window
                            const uint32_t jt01 = hw_u16(hw, src, jp) | (hw_u16(hw, src, jp + 2) << 16);
                            const uint32_t jt2 = hw_u16(hw, src, jp + 4);
                            if (COOP)
                                ok = coop_section(hufTl, hp, remain, litOut, (uint32_t)rs, jt01, jt2, S.coopCmd,
                                                  S.coopStg, P);
                            else if (S.job && last && noSeq &&
                                     huf_defer_section(S.job, hufTl, hp, remain, litOut, (uint32_t)rs, jt01, jt2)) {
                                ok = true;        // dec_huf_kernel decodes the streams (and reports their errors)
                                S.job = nullptr;  // one job per unit (a later frame of the unit decodes in place)
                            }
                            else
                                ok = huf_decode4_wave(hufTl, hp, remain, litOut, (uint32_t)rs, jt01, jt2, P);
                        }
                    }
                    if (ballot(!ok)) return z1::kDecErrHufStream;
                    P.mark(2);
                }
                wave_sync();
                if (noSeq) {
                    op += rs;
                } else {
                    // the sequences stage overlays sDec.tab: park the table if a later block may reuse it
                    if (!last && hufInLds && !hufParked) {
                        for (uint32_t i = (uint32_t)lane; i < (1u << hufTl); i += 64) gst<uint16_t>(S.htab + i, sDec.tab[i]);
                        hufParked = true;
                    }
                    hufInLds = false;
                    wave_sync();
                    const long r = exec_sequences_wave(seqSrc, seqSize, lit, rs, dst, op, dstCap, frameStart, S, last != 0, fs, P);
                    P.count(11);
                    if (r < 0) return r;
                    op = (size_t)r;
                    P.mark(4);
                }
                ip += bsize;
            }
            if (last) break;
        }
        if (fcsSize > 0 && (op - frameStart) != fcs) return z1::kDecErrCorrupt;
        if (checksum) {
            if (srcSize - ip < 4) return z1::kDecErrSrcSmall;
            ip += 4;
        }
    }
    wave_sync();
    return (long)op;
}

// ---------------------------------------------------------------------------------------------
// The batch decoder's fast path for the two frame shapes that make up most of a C5 chunk: a frame
// that is one raw block (the S and Llow streams) and a frame that is one compressed block of
// literals only with four Huffman streams and a new table (keys, M), whose streams are left to
// dec_huf_kernel as a job.  Everything is inlined into the kernel's unit loop: zstd_decompress_wave
// is a call, and at 96 VGPRs the call's spills, callee-saved registers and by-value arguments went
// through the wave's private stack -- ~120 KB of HBM writes per chunk (profiles/r04_*traffic*).
// Returns the decoded size, or -1 when the frame is anything else or anything is out of the
// ordinary (sizes, end of input, a table the job cannot hold): the caller then runs
// zstd_decompress_wave, which reaches the same result or reports the error, so statuses and bytes
// are the general decoder's in every case.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ long dec_frame_fast(const uint8_t* __restrict__ src, size_t srcSize, uint8_t* __restrict__ dst,
                                               size_t dstCap, uint8_t* job, uint16_t* htab, PhaseProf& P, HufBuildLds& H)
{
    if (srcSize < 9) return -1;
    HdrWin hw;
    hw_load(hw, src, srcSize, 0);
    if (hw_u32(hw, src, 0) != z1::kMagic) return -1;
    const uint32_t fhd = hw_byte(hw, src, 4);
    const unsigned checksum = (fhd >> 2) & 1, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
    if (fhd & 0x0B) return -1;  // reserved bit, or a dictionary id
    size_t ip = 5 + (singleSegment ? 0 : 1);
    const unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
    if (fcsSize == 8 || ip + fcsSize + 3 > srcSize) return -1;
    uint64_t fcs = 0;
    if (fcsSize == 1) fcs = hw_byte(hw, src, ip);
    else if (fcsSize == 2) fcs = (uint64_t)hw_u16(hw, src, ip) + 256;
    else if (fcsSize == 4) fcs = hw_u32(hw, src, ip);
    ip += fcsSize;
    const uint32_t bh = hw_u24(hw, src, ip);
    ip += 3;
    const size_t bsize = bh >> 3;
    const unsigned btype = (bh >> 1) & 3;
    P.mark(7);
    // one last block, and the frame (its checksum included) ends where the unit does
    if (!(bh & 1) || bsize > srcSize - ip || ip + bsize + (checksum ? 4 : 0) != srcSize) return -1;
    if (btype == z1::kBtRaw) {
        if (bsize > dstCap || (fcsSize > 0 && bsize != fcs)) return -1;
        wave_copy_nt(dst, src + ip, bsize);  // read by the merge only after the sections: non-temporal
        P.mark(5);
        return (long)bsize;
    }
    if (btype != z1::kBtCompressed || job == nullptr || bsize > z1::kMaxSrc || bsize < 5) return -1;
    const uint32_t lhc = hw_u32(hw, src, ip);
    const unsigned ltype = lhc & 3, sf = (lhc >> 2) & 3;
    if (ltype != z1::kSetCompressed || sf == 0) return -1;
    size_t lh, rs, cs;
    if (sf == 1) { lh = 3; rs = (lhc >> 4) & 0x3FF; cs = (lhc >> 14) & 0x3FF; }
    else if (sf == 2) { lh = 4; rs = (lhc >> 4) & 0x3FFF; cs = lhc >> 18; }
    else { lh = 5; rs = (lhc >> 4) & 0x3FFFF; cs = (lhc >> 22) + ((size_t)hw_byte(hw, src, ip + 4) << 10); }
    if (rs > z1::kMaxSrc || rs > dstCap || lh + cs + 1 != bsize || (fcsSize > 0 && rs != fcs)) return -1;
    if (hw_byte(hw, src, ip + lh + cs) != 0) return -1;  // the sequences section: none
    const uint8_t* hp = src + ip + lh;
    unsigned tl = 0, mn = 1;
    uint32_t kc[3] = {0, 0, 0};
    const size_t hsz = huf_build_dtable_body<true>(H, hp, cs, &tl, htab, &mn, &hw, (uint32_t)(ip + lh), &P, job + sizeof(HufJob), kc);
    P.mark(1);
    if (hsz == 0 || tl > kHufLdsLog || cs - hsz < 6) return -1;
    hp += hsz;
    const size_t remain = cs - hsz;
    const size_t jp = (size_t)(hp - src);
    const uint32_t jt01 = hw_u16(hw, src, jp) | (hw_u16(hw, src, jp + 2) << 16);
    const uint32_t jt2 = hw_u16(hw, src, jp + 4);
    if (!huf_defer_header(job, tl, hp, remain, dst, (uint32_t)rs, jt01, jt2, kc)) return -1;
    return (long)rs;
}

}  // namespace pgn
