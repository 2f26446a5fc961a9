// zstd1_common.h -- shared (host + device) building blocks of the zstd *level-1* frame format as
// produced by libzstd 1.4.8 / 1.4.9 `ZSTD_compress(dst, cap, src, n, 1)`, the call the reference's
// C5 codec makes once per stream (pgnano/svb16/C5.hpp:337,356,373,390,407; VBZ:
// signal_compression.cpp:65).  libzstd is a third-party dependency absent from the reference tree;
// the algorithm restated here is its published format (RFC 8878) plus the level-1 encoder
// decisions of that release line.  Every function is checked byte-for-byte against the real
// library by tests/test_zstd_model.py.
//
// These functions are the serial pieces that both the host model (zstd1_model.hip, test-only) and
// the GPU kernels (pgn_kernels.hip) run; the GPU replaces the data-parallel stages (match search,
// histograms, Huffman bit packing) with wave-parallel code of identical output.
//
// Parts of this file restate algorithms of Zstandard (libzstd 1.4.x), Copyright (c) 2016-present,
// Facebook, Inc., used under its BSD licence: see THIRD_PARTY_NOTICES.md at the repository root.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define PGN_HD __host__ __device__ inline

namespace pgn {
namespace z1 {

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr unsigned kHufTableLogDefault = 11;
constexpr unsigned kHufTableLogMax = 12;
constexpr unsigned kFseMinTableLog = 5;
constexpr unsigned kFseMaxTableLog = 12;
constexpr unsigned kLLFSELog = 9, kMLFSELog = 9, kOffFSELog = 8;
constexpr unsigned kMaxLL = 35, kMaxML = 52, kMaxOff = 31, kDefaultMaxOff = 28;
constexpr unsigned kLLDefaultNormLog = 6, kMLDefaultNormLog = 6, kOFDefaultNormLog = 5;
constexpr size_t kMaxSrc = 131072;        // ZSTD_BLOCKSIZE_MAX: one block (literals, sequences per block)

enum : unsigned { kSetBasic = 0, kSetRle = 1, kSetCompressed = 2, kSetRepeat = 3 };
enum : unsigned { kBtRaw = 0, kBtRle = 1, kBtCompressed = 2 };

// ---------------------------------------------------------------------------------------------
// Small tables (RFC 8878 3.1.1.3.2.1 / 4.1).  Kept as switch-free functions over constexpr arrays so
// the same code compiles for host and gfx950.
// ---------------------------------------------------------------------------------------------
PGN_HD unsigned ll_bits(unsigned code)
{
    static constexpr uint8_t t[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  1,  1,
                               1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[code];
}
PGN_HD unsigned ml_bits(unsigned code)
{
    static constexpr uint8_t t[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                               2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return t[code];
}
PGN_HD int16_t ll_default_norm(unsigned s)
{
    static constexpr int16_t t[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                               2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
    return t[s];
}
PGN_HD int16_t ml_default_norm(unsigned s)
{
    static constexpr int16_t t[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
    return t[s];
}
PGN_HD int16_t of_default_norm(unsigned s)
{
    static constexpr int16_t t[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    return t[s];
}
PGN_HD uint32_t ll_base(unsigned code)
{
    static constexpr uint32_t t[36] = {0,  1,  2,  3,  4,  5,   6,   7,   8,    9,    10,   11,
                                12, 13, 14, 15, 16, 18,  20,  22,  24,   28,   32,   40,
                                48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    return t[code];
}
PGN_HD uint32_t ml_base(unsigned code)  // match length (not mlBase): 3 + ...
{
    static constexpr uint32_t t[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                                17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30,
                                31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83,
                                99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
    return t[code];
}

PGN_HD unsigned highbit32(uint32_t v) { return 31u - (unsigned)__builtin_clz(v); }  // v != 0

PGN_HD unsigned ll_code(uint32_t litLength)
{
    static constexpr uint8_t t[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                               16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21,
                               22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                               24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
    return (litLength > 63) ? highbit32(litLength) + 19u : t[litLength];
}
PGN_HD unsigned ml_code(uint32_t mlBase)
{
    if (mlBase > 127) return highbit32(mlBase) + 36u;
    if (mlBase < 32) return mlBase;
    if (mlBase < 40) return 32u + ((mlBase - 32u) >> 1);
    if (mlBase < 48) return 36u + ((mlBase - 40u) >> 2);
    if (mlBase < 64) return 38u + ((mlBase - 48u) >> 3);
    if (mlBase < 96) return 40u + ((mlBase - 64u) >> 4);
    return 42u;
}

// ---------------------------------------------------------------------------------------------
// Level-1 compression parameters: row `level 1` of the four srcSize tiers of
// ZSTD_defaultCParameters, then ZSTD_adjustCParams_internal (window shrunk to the source,
// hashLog <= windowLog + 1, windowLog >= 10); equal to libzstd 1.4.8/1.4.9's
// ZSTD_getCParams(1, srcSize, 0) for every size (tests/test_zstd_model.py).
// ---------------------------------------------------------------------------------------------
struct Params {
    unsigned windowLog, hashLog, mls;
};
PGN_HD Params level1_params(size_t srcSize)
{
    Params p;
    if (srcSize <= 16384) { p.windowLog = 14; p.hashLog = 15; p.mls = 5; }
    else if (srcSize <= 131072) { p.windowLog = 17; p.hashLog = 13; p.mls = 6; }
    else if (srcSize <= 262144) { p.windowLog = 18; p.hashLog = 14; p.mls = 6; }
    else { p.windowLog = 19; p.hashLog = 14; p.mls = 7; }
    unsigned srcLog = (srcSize < 64) ? 6u : highbit32((uint32_t)(srcSize - 1)) + 1u;
    if (p.windowLog > srcLog) p.windowLog = srcLog;
    if (p.hashLog > p.windowLog + 1) p.hashLog = p.windowLog + 1;
    if (p.windowLog < 10) p.windowLog = 10;
    return p;
}

PGN_HD size_t compress_bound(size_t n)  // ZSTD_compressBound
{
    return n + (n >> 8) + ((n < (128u << 10)) ? (((128u << 10) - n) >> 11) : 0u);
}

PGN_HD uint32_t rd32(const uint8_t* p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
PGN_HD uint64_t rd64(const uint8_t* p)
{
    return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}
PGN_HD void wr16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
PGN_HD void wr24(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); }
PGN_HD void wr32(uint8_t* p, uint32_t v) { wr16(p, v); wr16(p + 2, v >> 16); }

// ZSTD_hashPtr for mls 5 / 6 / 7 of the 8-byte little-endian word at a position.
PGN_HD uint32_t hash_word(uint64_t v, unsigned hlog, unsigned mls)
{
    if (mls == 5) return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - hlog));
    if (mls == 6) return (uint32_t)(((v << 16) * 227718039650203ull) >> (64 - hlog));
    return (uint32_t)(((v << 8) * 58295818150454627ull) >> (64 - hlog));
}
PGN_HD uint32_t hash_at(const uint8_t* p, unsigned hlog, unsigned mls) { return hash_word(rd64(p), hlog, mls); }

// ---------------------------------------------------------------------------------------------
// Frame header (ZSTD_writeFrameHeader: content size present, no checksum / dictID; single segment
// when the window covers the source, else a window descriptor byte (windowLog - 10) << 3)
// ---------------------------------------------------------------------------------------------
PGN_HD size_t write_frame_header(uint8_t* op, size_t srcSize, unsigned windowLog)
{
    wr32(op, kMagic);
    const unsigned single = ((size_t)1 << windowLog) >= srcSize;
    unsigned fcsCode = (srcSize >= 256) + (srcSize >= 65536 + 256) + (srcSize >= 0xFFFFFFFFull);
    op[4] = (uint8_t)((single << 5) + (fcsCode << 6));
    size_t pos = 5;
    if (!single) op[pos++] = (uint8_t)((windowLog - 10u) << 3);
    switch (fcsCode) {
    case 0: op[pos] = (uint8_t)srcSize; return pos + 1;
    case 1: wr16(op + pos, (uint32_t)(srcSize - 256)); return pos + 2;
    default: wr32(op + pos, (uint32_t)srcSize); return pos + 4;
    }
}
PGN_HD size_t frame_header_size(size_t srcSize, unsigned windowLog)
{
    unsigned fcsCode = (srcSize >= 256) + (srcSize >= 65536 + 256);
    return (fcsCode == 0 ? 6 : (fcsCode == 1 ? 7 : 9)) + (((size_t)1 << windowLog) < srcSize);
}
// ZSTD_getLowestPrefixIndex(ms, end index, windowLog) of a frame (dictLimit 1, no dictionary): the
// lowest index a match candidate of a block ending at position `end` may exceed.
PGN_HD uint32_t window_low_index(size_t end, unsigned windowLog)
{
    const size_t maxDist = (size_t)1 << windowLog;
    return end > maxDist ? (uint32_t)(end + 1 - maxDist) : 1u;
}

// Literal section headers (ZSTD_noCompressLiterals / ZSTD_compressRleLiteralsBlock).
PGN_HD size_t raw_lit_header_size(size_t n) { return 1 + (n > 31) + (n > 4095); }
PGN_HD size_t write_rawrle_lit_header(uint8_t* op, size_t n, unsigned type)
{
    size_t fl = raw_lit_header_size(n);
    if (fl == 1) op[0] = (uint8_t)(type + (n << 3));
    else if (fl == 2) wr16(op, (uint32_t)(type + (1u << 2) + (n << 4)));
    else wr24(op, (uint32_t)(type + (3u << 2) + (n << 4)));
    return fl;
}
PGN_HD size_t huf_lit_header_size(size_t n) { return 3 + (n >= 1024) + (n >= 16384); }
// hType: kSetCompressed (a new table) or kSetRepeat (the previous block's table, "treeless")
PGN_HD void write_huf_lit_header(uint8_t* op, size_t lhSize, size_t srcSize, size_t cLitSize, bool singleStream,
                                 unsigned hType = kSetCompressed)
{
    if (lhSize == 3) {
        wr24(op, (uint32_t)(hType + ((!singleStream) << 2) + (srcSize << 4) + (cLitSize << 14)));
    } else if (lhSize == 4) {
        wr32(op, (uint32_t)(hType + (2u << 2) + (srcSize << 4) + (cLitSize << 18)));
    } else {
        wr32(op, (uint32_t)(hType + (3u << 2) + (srcSize << 4) + (cLitSize << 22)));
        op[4] = (uint8_t)(cLitSize >> 10);
    }
}

// ---------------------------------------------------------------------------------------------
// Little-endian forward bit writer (BIT_CStream semantics without the overflow policy: the
// callers size the destination from exact bit counts).
// ---------------------------------------------------------------------------------------------
struct BitW {
    uint8_t* p;
    uint64_t acc;
    unsigned n;  // bits in acc
};
PGN_HD void bw_init(BitW& b, uint8_t* dst) { b.p = dst; b.acc = 0; b.n = 0; }
PGN_HD void bw_add(BitW& b, uint64_t v, unsigned nb)
{
    if (nb == 0) return;
    v &= (nb >= 64) ? ~0ull : ((1ull << nb) - 1);
    b.acc |= v << b.n;
    b.n += nb;
    while (b.n >= 8) { *b.p++ = (uint8_t)b.acc; b.acc >>= 8; b.n -= 8; }
}
// BIT_closeCStream: end mark then flush; returns bytes written since `start`.
PGN_HD size_t bw_close(BitW& b, const uint8_t* start)
{
    bw_add(b, 1, 1);
    if (b.n) { *b.p++ = (uint8_t)b.acc; b.acc = 0; b.n = 0; }
    return (size_t)(b.p - start);
}

// ---------------------------------------------------------------------------------------------
// FSE (finite state entropy) encoder pieces: FSE_optimalTableLog, FSE_normalizeCount (+M2),
// FSE_writeNCount, FSE_buildCTable.
// ---------------------------------------------------------------------------------------------
PGN_HD unsigned fse_min_table_log(size_t srcSize, unsigned maxSymbolValue)
{
    unsigned minBitsSrc = highbit32((uint32_t)srcSize) + 1;
    unsigned minBitsSymbols = highbit32(maxSymbolValue) + 2;
    return minBitsSrc < minBitsSymbols ? minBitsSrc : minBitsSymbols;
}
PGN_HD unsigned fse_optimal_table_log(unsigned maxTableLog, size_t srcSize, unsigned maxSymbolValue, unsigned minus)
{
    unsigned maxBitsSrc = highbit32((uint32_t)(srcSize - 1)) - minus;
    unsigned tableLog = maxTableLog;
    unsigned minBits = fse_min_table_log(srcSize, maxSymbolValue);
    if (tableLog == 0) tableLog = 11;
    if (maxBitsSrc < tableLog) tableLog = maxBitsSrc;
    if (minBits > tableLog) tableLog = minBits;
    if (tableLog < kFseMinTableLog) tableLog = kFseMinTableLog;
    if (tableLog > kFseMaxTableLog) tableLog = kFseMaxTableLog;
    return tableLog;
}

// returns false on error
PGN_HD bool fse_normalize_m2(int16_t* norm, unsigned tableLog, const uint32_t* count, size_t total,
                             unsigned maxSymbolValue, int16_t lowProbCount)
{
    const int16_t NOT_YET = -2;
    uint32_t distributed = 0;
    uint32_t lowThreshold = (uint32_t)(total >> tableLog);
    uint32_t lowOne = (uint32_t)((total * 3) >> (tableLog + 1));
    for (unsigned s = 0; s <= maxSymbolValue; s++) {
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) { norm[s] = lowProbCount; distributed++; total -= count[s]; continue; }
        if (count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
        norm[s] = NOT_YET;
    }
    uint32_t toDistribute = (1u << tableLog) - distributed;
    if (toDistribute == 0) return true;
    if ((total / toDistribute) > lowOne) {
        lowOne = (uint32_t)((total * 3) / (toDistribute * 2));
        for (unsigned s = 0; s <= maxSymbolValue; s++) {
            if ((norm[s] == NOT_YET) && (count[s] <= lowOne)) {
                norm[s] = 1; distributed++; total -= count[s];
            }
        }
        toDistribute = (1u << tableLog) - distributed;
    }
    if (distributed == maxSymbolValue + 1) {
        unsigned maxV = 0;
        uint32_t maxC = 0;
        for (unsigned s = 0; s <= maxSymbolValue; s++)
            if (count[s] > maxC) { maxV = s; maxC = count[s]; }
        norm[maxV] = (int16_t)(norm[maxV] + toDistribute);
        return true;
    }
    if (total == 0) {
        for (unsigned s = 0; toDistribute > 0; s = (s + 1) % (maxSymbolValue + 1))
            if (norm[s] > 0) { toDistribute--; norm[s]++; }
        return true;
    }
    {
        uint64_t vStepLog = 62 - tableLog;
        uint64_t mid = (1ull << (vStepLog - 1)) - 1;
        uint64_t rStep = ((((uint64_t)1 << vStepLog) * toDistribute) + mid) / (uint32_t)total;
        uint64_t tmpTotal = mid;
        for (unsigned s = 0; s <= maxSymbolValue; s++) {
            if (norm[s] == NOT_YET) {
                uint64_t end = tmpTotal + (count[s] * rStep);
                uint32_t sStart = (uint32_t)(tmpTotal >> vStepLog);
                uint32_t sEnd = (uint32_t)(end >> vStepLog);
                uint32_t weight = sEnd - sStart;
                if (weight < 1) return false;
                norm[s] = (int16_t)weight;
                tmpTotal = end;
            }
        }
    }
    return true;
}

// FSE_normalizeCount; returns false on error.  useLowProbCount as in libzstd 1.4.7+.
PGN_HD bool fse_normalize(int16_t* norm, unsigned tableLog, const uint32_t* count, size_t total,
                          unsigned maxSymbolValue, bool useLowProbCount)
{
    if (tableLog < kFseMinTableLog || tableLog > kFseMaxTableLog) return false;
    if (tableLog < fse_min_table_log(total, maxSymbolValue)) return false;
    constexpr uint32_t rtbTable[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    const int16_t lowProbCount = useLowProbCount ? -1 : 1;
    const uint64_t scale = 62 - tableLog;
    const uint64_t step = ((uint64_t)1 << 62) / total;
    const uint64_t vStep = 1ull << (scale - 20);
    int stillToDistribute = 1 << tableLog;
    unsigned largest = 0;
    int16_t largestP = 0;
    uint32_t lowThreshold = (uint32_t)(total >> tableLog);
    for (unsigned s = 0; s <= maxSymbolValue; s++) {
        if (count[s] == total) return false;  // rle: callers never get here
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) {
            norm[s] = lowProbCount;
            stillToDistribute--;
        } else {
            int16_t proba = (int16_t)((count[s] * step) >> scale);
            if (proba < 8) {
                uint64_t restToBeat = vStep * rtbTable[proba];
                proba += (int16_t)((count[s] * step) - ((uint64_t)proba << scale) > restToBeat);
            }
            if (proba > largestP) { largestP = proba; largest = s; }
            norm[s] = proba;
            stillToDistribute -= proba;
        }
    }
    if (-stillToDistribute >= (norm[largest] >> 1)) {
        return fse_normalize_m2(norm, tableLog, count, total, maxSymbolValue, lowProbCount);
    }
    norm[largest] = (int16_t)(norm[largest] + stillToDistribute);
    return true;
}

// FSE_writeNCount; returns bytes written, 0 on error.
PGN_HD size_t fse_write_ncount(uint8_t* out0, const int16_t* norm, unsigned maxSymbolValue, unsigned tableLog)
{
    uint8_t* out = out0;
    const int tableSize = 1 << tableLog;
    uint32_t bitStream = 0;
    int bitCount = 0;
    unsigned symbol = 0;
    const unsigned alphabetSize = maxSymbolValue + 1;
    int previousIs0 = 0;
    bitStream += (tableLog - kFseMinTableLog) << bitCount;
    bitCount += 4;
    int remaining = tableSize + 1;
    int threshold = tableSize;
    int nbBits = (int)tableLog + 1;
    while ((symbol < alphabetSize) && (remaining > 1)) {
        if (previousIs0) {
            unsigned start = symbol;
            while ((symbol < alphabetSize) && !norm[symbol]) symbol++;
            if (symbol == alphabetSize) break;
            while (symbol >= start + 24) {
                start += 24;
                bitStream += 0xFFFFu << bitCount;
                out[0] = (uint8_t)bitStream;
                out[1] = (uint8_t)(bitStream >> 8);
                out += 2;
                bitStream >>= 16;
            }
            while (symbol >= start + 3) {
                start += 3;
                bitStream += 3u << bitCount;
                bitCount += 2;
            }
            bitStream += (symbol - start) << bitCount;
            bitCount += 2;
            if (bitCount > 16) {
                out[0] = (uint8_t)bitStream;
                out[1] = (uint8_t)(bitStream >> 8);
                out += 2;
                bitStream >>= 16;
                bitCount -= 16;
            }
        }
        {
            int count = norm[symbol++];
            const int max = (2 * threshold - 1) - remaining;
            remaining -= count < 0 ? -count : count;
            count++;
            if (count >= threshold) count += max;
            bitStream += (uint32_t)count << bitCount;
            bitCount += nbBits;
            bitCount -= (count < max);
            previousIs0 = (count == 1);
            if (remaining < 1) return 0;
            while (remaining < threshold) { nbBits--; threshold >>= 1; }
        }
        if (bitCount > 16) {
            out[0] = (uint8_t)bitStream;
            out[1] = (uint8_t)(bitStream >> 8);
            out += 2;
            bitStream >>= 16;
            bitCount -= 16;
        }
    }
    if (remaining != 1) return 0;
    out[0] = (uint8_t)bitStream;
    out[1] = (uint8_t)(bitStream >> 8);
    out += (bitCount + 7) / 8;
    return (size_t)(out - out0);
}

// FSE compression table: stateTable[tableSize] + per-symbol transform.
struct FseCTable {
    unsigned tableLog;
    uint16_t stateTable[1 << kLLFSELog];  // 512 >= any table used here (<= 2^9)
    uint32_t deltaNbBits[kMaxML + 1];
    int32_t deltaFindState[kMaxML + 1];
};

// FSE_buildCTable_wksp.  `tableSymbol` scratch: >= 2^tableLog bytes.
PGN_HD void fse_build_ctable(FseCTable& ct, const int16_t* norm, unsigned maxSymbolValue, unsigned tableLog,
                             uint8_t* tableSymbol)
{
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t tableMask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    uint32_t cumul[kMaxML + 2];
    uint32_t highThreshold = tableSize - 1;
    ct.tableLog = tableLog;
    cumul[0] = 0;
    for (unsigned u = 1; u <= maxSymbolValue + 1; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            tableSymbol[highThreshold--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
        }
    }
    cumul[maxSymbolValue + 1] = tableSize + 1;
    {
        uint32_t position = 0;
        for (unsigned symbol = 0; symbol <= maxSymbolValue; symbol++) {
            int freq = norm[symbol];
            for (int k = 0; k < freq; k++) {
                tableSymbol[position] = (uint8_t)symbol;
                position = (position + step) & tableMask;
                while (position > highThreshold) position = (position + step) & tableMask;
            }
        }
    }
    for (uint32_t u = 0; u < tableSize; u++) {
        uint8_t s = tableSymbol[u];
        ct.stateTable[cumul[s]++] = (uint16_t)(tableSize + u);
    }
    unsigned total = 0;
    for (unsigned s = 0; s <= maxSymbolValue; s++) {
        switch (norm[s]) {
        case 0:
            ct.deltaNbBits[s] = ((tableLog + 1) << 16) - (1u << tableLog);
            ct.deltaFindState[s] = 0;
            break;
        case -1:
        case 1:
            ct.deltaNbBits[s] = (tableLog << 16) - (1u << tableLog);
            ct.deltaFindState[s] = (int32_t)total - 1;
            total++;
            break;
        default: {
            uint32_t maxBitsOut = tableLog - highbit32((uint32_t)(norm[s] - 1));
            uint32_t minStatePlus = (uint32_t)norm[s] << maxBitsOut;
            ct.deltaNbBits[s] = (maxBitsOut << 16) - minStatePlus;
            ct.deltaFindState[s] = (int32_t)total - norm[s];
            total += (unsigned)norm[s];
        }
        }
    }
}
// FSE_buildCTable_rle: tableLog 0, every symbol emits 0 bits.
PGN_HD void fse_build_ctable_rle(FseCTable& ct, unsigned symbol)
{
    ct.tableLog = 0;
    ct.stateTable[0] = 0;
    ct.stateTable[1] = 0;
    ct.deltaNbBits[symbol] = 0;
    ct.deltaFindState[symbol] = 0;
}

struct FseState {
    uint32_t value;
};
PGN_HD void fse_init_state2(FseState& st, const FseCTable& ct, unsigned symbol)
{
    uint32_t nbBitsOut = (ct.deltaNbBits[symbol] + (1u << 15)) >> 16;
    uint32_t v = (nbBitsOut << 16) - ct.deltaNbBits[symbol];
    st.value = ct.stateTable[(v >> nbBitsOut) + ct.deltaFindState[symbol]];
}
PGN_HD void fse_encode(BitW& bw, FseState& st, const FseCTable& ct, unsigned symbol)
{
    uint32_t nbBitsOut = (st.value + ct.deltaNbBits[symbol]) >> 16;
    bw_add(bw, st.value, nbBitsOut);
    st.value = ct.stateTable[(st.value >> nbBitsOut) + ct.deltaFindState[symbol]];
}
PGN_HD void fse_flush(BitW& bw, const FseState& st, const FseCTable& ct) { bw_add(bw, st.value, ct.tableLog); }

// ---------------------------------------------------------------------------------------------
// Huffman (HUF_buildCTable_wksp + HUF_setMaxHeight + HUF_writeCTable)
// ---------------------------------------------------------------------------------------------
struct HufNode {
    uint32_t count;
    uint16_t parent;
    uint8_t byte;
    uint8_t nbBits;
};
constexpr int kHufStartNode = 256;  // HUF_SYMBOLVALUE_MAX + 1

// Stable sort by decreasing count (HUF_sort: rank buckets + insertion; equivalent to sorting by
// (count desc, symbol asc)).  nodes: huffNode (huffNode0 + 1), 512 entries.
PGN_HD void huf_sort_serial(HufNode* huffNode, const uint32_t* count, unsigned maxSymbolValue)
{
    unsigned pos = 0;
    // counting by rank buckets of highbit(count+1), largest first, then insertion within bucket
    uint32_t rankBase[33], rankCur[33];
    for (int r = 0; r < 33; r++) rankBase[r] = 0;
    for (unsigned n = 0; n <= maxSymbolValue; n++) rankBase[highbit32(count[n] + 1)]++;
    // bucket r starts after all buckets > r
    uint32_t acc = 0;
    for (int r = 32; r >= 0; r--) { uint32_t c = rankBase[r]; rankBase[r] = acc; acc += c; }
    for (int r = 0; r < 33; r++) rankCur[r] = rankBase[r];
    for (unsigned n = 0; n <= maxSymbolValue; n++) {
        uint32_t c = count[n];
        unsigned r = highbit32(c + 1);
        pos = rankCur[r]++;
        while ((pos > rankBase[r]) && (c > huffNode[pos - 1].count)) {
            huffNode[pos] = huffNode[pos - 1];
            pos--;
        }
        huffNode[pos].count = c;
        huffNode[pos].byte = (uint8_t)n;
    }
}

// HUF_setMaxHeight.  Returns the enforced max number of bits.
PGN_HD unsigned huf_set_max_height(HufNode* huffNode, unsigned lastNonNull, unsigned maxNbBits)
{
    const unsigned largestBits = huffNode[lastNonNull].nbBits;
    if (largestBits <= maxNbBits) return largestBits;
    int totalCost = 0;
    const unsigned baseCost = 1u << (largestBits - maxNbBits);
    int n = (int)lastNonNull;
    while (huffNode[n].nbBits > maxNbBits) {
        totalCost += (int)(baseCost - (1u << (largestBits - huffNode[n].nbBits)));
        huffNode[n].nbBits = (uint8_t)maxNbBits;
        n--;
    }
    while (huffNode[n].nbBits == maxNbBits) n--;
    totalCost >>= (largestBits - maxNbBits);
    {
        const uint32_t noSymbol = 0xF0F0F0F0u;
        uint32_t rankLast[kHufTableLogMax + 2];
        for (int i = 0; i < (int)kHufTableLogMax + 2; i++) rankLast[i] = noSymbol;
        {
            unsigned currentNbBits = maxNbBits;
            for (int pos = n; pos >= 0; pos--) {
                if (huffNode[pos].nbBits >= currentNbBits) continue;
                currentNbBits = huffNode[pos].nbBits;
                rankLast[maxNbBits - currentNbBits] = (uint32_t)pos;
            }
        }
        while (totalCost > 0) {
            unsigned nBitsToDecrease = highbit32((uint32_t)totalCost) + 1;
            for (; nBitsToDecrease > 1; nBitsToDecrease--) {
                uint32_t highPos = rankLast[nBitsToDecrease];
                uint32_t lowPos = rankLast[nBitsToDecrease - 1];
                if (highPos == noSymbol) continue;
                if (lowPos == noSymbol) break;
                {
                    uint32_t highTotal = huffNode[highPos].count;
                    uint32_t lowTotal = 2 * huffNode[lowPos].count;
                    if (highTotal <= lowTotal) break;
                }
            }
            while ((nBitsToDecrease <= kHufTableLogMax) && (rankLast[nBitsToDecrease] == noSymbol))
                nBitsToDecrease++;
            totalCost -= 1 << (nBitsToDecrease - 1);
            if (rankLast[nBitsToDecrease - 1] == noSymbol)
                rankLast[nBitsToDecrease - 1] = rankLast[nBitsToDecrease];
            huffNode[rankLast[nBitsToDecrease]].nbBits++;
            if (rankLast[nBitsToDecrease] == 0) {
                rankLast[nBitsToDecrease] = noSymbol;
            } else {
                rankLast[nBitsToDecrease]--;
                if (huffNode[rankLast[nBitsToDecrease]].nbBits != maxNbBits - nBitsToDecrease)
                    rankLast[nBitsToDecrease] = noSymbol;
            }
        }
        while (totalCost < 0) {
            if (rankLast[1] == noSymbol) {
                while (huffNode[n].nbBits == maxNbBits) n--;
                huffNode[n + 1].nbBits--;
                rankLast[1] = (uint32_t)(n + 1);
                totalCost++;
                continue;
            }
            huffNode[rankLast[1] + 1].nbBits--;
            rankLast[1]++;
            totalCost++;
        }
    }
    return maxNbBits;
}

// HUF_buildCTable_wksp given the sorted node array (huffNode = huffNode0 + 1, huffNode0 has 512+
// entries zeroed beyond the sorted symbols).  Fills nbBits[] and val[] per symbol
// (0..maxSymbolValue) and returns maxNbBits.
PGN_HD unsigned huf_build_from_sorted(HufNode* huffNode0, unsigned maxSymbolValue, unsigned maxNbBits,
                                      uint8_t* nbBitsOut, uint16_t* valOut)
{
    HufNode* huffNode = huffNode0 + 1;
    int nodeNb = kHufStartNode;
    int nonNullRank = (int)maxSymbolValue;
    while (huffNode[nonNullRank].count == 0) nonNullRank--;
    int lowS = nonNullRank;
    int nodeRoot = nodeNb + lowS - 1;
    int lowN = nodeNb;
    huffNode[nodeNb].count = huffNode[lowS].count + huffNode[lowS - 1].count;
    huffNode[lowS].parent = huffNode[lowS - 1].parent = (uint16_t)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int n = nodeNb; n <= nodeRoot; n++) huffNode[n].count = 1u << 30;
    huffNode0[0].count = 1u << 31;
    while (nodeNb <= nodeRoot) {
        int n1 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        int n2 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        huffNode[nodeNb].count = huffNode[n1].count + huffNode[n2].count;
        huffNode[n1].parent = huffNode[n2].parent = (uint16_t)nodeNb;
        nodeNb++;
    }
    huffNode[nodeRoot].nbBits = 0;
    for (int n = nodeRoot - 1; n >= kHufStartNode; n--)
        huffNode[n].nbBits = (uint8_t)(huffNode[huffNode[n].parent].nbBits + 1);
    for (int n = 0; n <= nonNullRank; n++)
        huffNode[n].nbBits = (uint8_t)(huffNode[huffNode[n].parent].nbBits + 1);
    maxNbBits = huf_set_max_height(huffNode, (unsigned)nonNullRank, maxNbBits);
    uint16_t nbPerRank[kHufTableLogMax + 1];
    uint16_t valPerRank[kHufTableLogMax + 1];
    for (unsigned i = 0; i <= kHufTableLogMax; i++) { nbPerRank[i] = 0; valPerRank[i] = 0; }
    for (int n = 0; n <= nonNullRank; n++) nbPerRank[huffNode[n].nbBits]++;
    {
        uint16_t mn = 0;
        for (int n = (int)maxNbBits; n > 0; n--) {
            valPerRank[n] = mn;
            mn = (uint16_t)(mn + nbPerRank[n]);
            mn >>= 1;
        }
    }
    for (int n = 0; n <= (int)maxSymbolValue; n++) nbBitsOut[huffNode[n].byte] = huffNode[n].nbBits;
    for (int n = 0; n <= (int)maxSymbolValue; n++) valOut[n] = valPerRank[nbBitsOut[n]]++;
    return maxNbBits;
}

// HUF_compressWeights (FSE, tableLog <= 6) -- returns size, 0 = not compressible, 1 = rle.
// scratch: >= 64 bytes; ct workspace provided by the caller.
PGN_HD size_t huf_compress_weights(uint8_t* dst, const uint8_t* weights, unsigned wtSize, FseCTable& ct, uint8_t* scratch)
{
    if (wtSize <= 1) return 0;
    uint32_t count[kHufTableLogMax + 1];
    for (unsigned i = 0; i <= kHufTableLogMax; i++) count[i] = 0;
    for (unsigned i = 0; i < wtSize; i++) count[weights[i]]++;
    unsigned maxSymbolValue = kHufTableLogMax;
    while (!count[maxSymbolValue]) maxSymbolValue--;
    uint32_t maxCount = 0;
    for (unsigned s = 0; s <= maxSymbolValue; s++) if (count[s] > maxCount) maxCount = count[s];
    if (maxCount == wtSize) return 1;
    if (maxCount == 1) return 0;
    unsigned tableLog = fse_optimal_table_log(6, wtSize, maxSymbolValue, 2);
    int16_t norm[kHufTableLogMax + 1];
    if (!fse_normalize(norm, tableLog, count, wtSize, maxSymbolValue, false)) return 0;
    size_t hSize = fse_write_ncount(dst, norm, maxSymbolValue, tableLog);
    if (hSize == 0) return 0;
    fse_build_ctable(ct, norm, maxSymbolValue, tableLog, scratch);
    // FSE_compress_usingCTable (two interleaved states), srcSize > 2 here
    if (wtSize <= 2) return 0;
    uint8_t* op = dst + hSize;
    BitW bw;
    bw_init(bw, op);
    const uint8_t* ip = weights + wtSize;
    FseState s1, s2;
    size_t srcSize = wtSize;
    if (srcSize & 1) {
        fse_init_state2(s1, ct, *--ip);
        fse_init_state2(s2, ct, *--ip);
        fse_encode(bw, s1, ct, *--ip);
    } else {
        fse_init_state2(s2, ct, *--ip);
        fse_init_state2(s1, ct, *--ip);
    }
    srcSize -= 2;
    if (srcSize & 2) {
        fse_encode(bw, s2, ct, *--ip);
        fse_encode(bw, s1, ct, *--ip);
    }
    while (ip > weights) {
        fse_encode(bw, s2, ct, *--ip);
        fse_encode(bw, s1, ct, *--ip);
        fse_encode(bw, s2, ct, *--ip);
        fse_encode(bw, s1, ct, *--ip);
    }
    fse_flush(bw, s2, ct);
    fse_flush(bw, s1, ct);
    size_t cSize = bw_close(bw, op);
    return hSize + cSize;
}

// HUF_writeCTable.  Returns header size; 0 = error (raw weights impossible: maxSymbolValue > 128).
PGN_HD size_t huf_write_ctable(uint8_t* op, const uint8_t* nbBits, unsigned maxSymbolValue, unsigned huffLog,
                               FseCTable& ct, uint8_t* scratch)
{
    uint8_t huffWeight[256];
    uint8_t bitsToWeight[kHufTableLogMax + 1];
    bitsToWeight[0] = 0;
    for (unsigned n = 1; n < huffLog + 1; n++) bitsToWeight[n] = (uint8_t)(huffLog + 1 - n);
    for (unsigned n = 0; n < maxSymbolValue; n++) huffWeight[n] = bitsToWeight[nbBits[n]];
    size_t hSize = huf_compress_weights(op + 1, huffWeight, maxSymbolValue, ct, scratch);
    if ((hSize > 1) & (hSize < maxSymbolValue / 2)) {
        op[0] = (uint8_t)hSize;
        return hSize + 1;
    }
    if (maxSymbolValue > (256 - 128)) return 0;
    op[0] = (uint8_t)(128 + (maxSymbolValue - 1));
    huffWeight[maxSymbolValue] = 0;
    for (unsigned n = 0; n < maxSymbolValue; n += 2)
        op[(n / 2) + 1] = (uint8_t)((huffWeight[n] << 4) + huffWeight[n + 1]);
    return ((maxSymbolValue + 1) / 2) + 1;
}

// HUF_optimalTableLog (FSE_optimalTableLog_internal with minus = 1)
PGN_HD unsigned huf_optimal_table_log(unsigned maxTableLog, size_t srcSize, unsigned maxSymbolValue)
{
    return fse_optimal_table_log(maxTableLog, srcSize, maxSymbolValue, 1);
}

// ---------------------------------------------------------------------------------------------
// Sequences
// ---------------------------------------------------------------------------------------------
struct Seq {
    uint32_t litLength;  // full literal length
    uint32_t offset;     // stored offset value: offCode + 1 (1 = repcode 0, else distance + 3)
    uint32_t mlBase;     // match length - 3
};

// ZSTD_selectEncodingType for strategy ZSTD_fast (< ZSTD_lazy), first block (repeat none).
PGN_HD unsigned select_encoding_type(size_t mostFrequent, size_t nbSeq, unsigned defaultNormLog, bool defaultAllowed)
{
    if (mostFrequent == nbSeq) {
        if (defaultAllowed && nbSeq <= 2) return kSetBasic;
        return kSetRle;
    }
    if (defaultAllowed) {
        const size_t mult = 10 - 1;  // strategy fast = 1
        const size_t dynamicFse_nbSeq_min = (((size_t)1 << defaultNormLog) * mult) >> 3;
        if ((nbSeq < dynamicFse_nbSeq_min) || (mostFrequent < (nbSeq >> (defaultNormLog - 1)))) return kSetBasic;
    }
    return kSetCompressed;
}

}  // namespace z1
}  // namespace pgn
