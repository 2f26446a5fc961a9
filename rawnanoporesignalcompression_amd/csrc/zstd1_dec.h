// zstd1_dec.h -- zstd frame decoder written from the format specification (RFC 8878), used where
// the reference calls ZSTD_getFrameContentSize / ZSTD_decompress (C5.hpp:493-667,
// signal_compression.cpp:100-118).  Host + device; every stage is serial except the four Huffman
// streams, which the GPU decodes on four lanes (huf_decode_stream is called per stream).
//
// Scope: everything ZSTD_decompress accepts without a dictionary -- concatenated and skippable
// frames, raw / RLE / compressed blocks, raw / RLE / Huffman / treeless literals, predefined / RLE /
// FSE / repeat sequence tables, repeat offsets, optional content checksum (skipped).
//
// Parts of this file restate algorithms of Zstandard (libzstd 1.4.x), Copyright (c) 2016-present,
// Facebook, Inc., used under its BSD licence: see THIRD_PARTY_NOTICES.md at the repository root.
#pragma once
#include "zstd1_common.h"

namespace pgn {
namespace z1 {

enum DecErr : int {
    kDecOk = 0,
    kDecErrHeader = -1,     // not a zstd frame / unsupported header
    kDecErrCorrupt = -2,    // malformed block content
    kDecErrDstSmall = -3,   // output larger than the capacity given
    kDecErrSrcSmall = -4,   // truncated input
    kDecErrHufTable = -5,   // malformed Huffman table description
    kDecErrHufStream = -6,  // malformed Huffman stream
};

// ---------------------------------------------------------------------------------------------
// ZSTD_getFrameContentSize semantics: returns content size; *ok = false when unknown / error
// (the reference maps both to "Input data not compressed by zstd").
// ---------------------------------------------------------------------------------------------
PGN_HD uint64_t frame_content_size(const uint8_t* src, size_t n, bool* ok)
{
    *ok = false;
    if (n < 4) return 0;
    uint32_t magic = rd32(src);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame: content size 0
        if (n < 8) return 0;
        *ok = true;
        return 0;
    }
    if (magic != kMagic) return 0;
    if (n < 5) return 0;
    uint8_t fhd = src[4];
    unsigned dictIDFlag = fhd & 3, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
    if (fhd & 0x08) return 0;  // reserved bit
    size_t pos = 5 + !singleSegment;
    const unsigned didSize[4] = {0, 1, 2, 4};
    pos += didSize[dictIDFlag];
    unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
    if (n < pos + fcsSize) return 0;
    if (fcsSize == 0) return 0;  // unknown
    uint64_t v;
    switch (fcsSize) {
    case 1: v = src[pos]; break;
    case 2: v = (uint64_t)(src[pos] | (src[pos + 1] << 8)) + 256; break;
    case 4: v = rd32(src + pos); break;
    default: v = rd64(src + pos); break;
    }
    *ok = true;
    return v;
}

// An upper bound on the bytes ZSTD_decompress can produce from the first frame of src[0, n): the
// frame's blocks are walked by their headers -- a raw or RLE block its size, a compressed block the
// regenerated size of its literals when its sequence count is 0, else ZSTD_BLOCKSIZE_MAX (128 KiB).
// -1: the first frame cannot decode at all (not a frame, a reserved block type, a block past n),
// which libzstd reports as an error.  A skippable frame produces nothing.  Used only for frames whose
// content size claims more than the decoder's buffers hold: a claim above the bound fails the
// frame-content-size check of ZSTD_decompress (or the frame fails before it), whatever follows.
PGN_HD int64_t frame_content_bound(const uint8_t* src, size_t n)
{
    if (n < 5) return -1;
    const uint32_t magic = rd32(src);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) return 0;
    if (magic != kMagic) return -1;
    const uint8_t fhd = src[4];
    const unsigned dictIDFlag = fhd & 3, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
    const unsigned didSize[4] = {0, 1, 2, 4};
    const unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
    size_t pos = 5 + !singleSegment + didSize[dictIDFlag] + fcsSize;
    if (pos > n) return -1;
    int64_t bound = 0;
    while (true) {
        if (n - pos < 3) return -1;
        const uint32_t bh = (uint32_t)src[pos] | ((uint32_t)src[pos + 1] << 8) | ((uint32_t)src[pos + 2] << 16);
        pos += 3;
        const uint32_t type = (bh >> 1) & 3u, bsize = bh >> 3;
        if (type == 3) return -1;
        if (type == 1) {  // RLE: one byte, bsize copies
            if (n - pos < 1) return -1;
            pos += 1;
            bound += bsize;
        } else {
            if (n - pos < bsize) return -1;
            if (type == 0) {
                bound += bsize;
            } else {  // compressed: literals header (RFC 8878 3.1.1.3.1.1), then the sequence count byte
                const uint8_t* b = src + pos;
                int64_t cb = 131072;
                if (bsize >= 1) {
                    const uint32_t lt = b[0] & 3u, sf = (b[0] >> 2) & 3u;
                    uint32_t lh = 0, regen = 0, comp = 0;
                    if (lt < 2) {
                        lh = sf == 1 ? 2 : (sf == 3 ? 3 : 1);
                        if (bsize >= lh) {
                            regen = sf == 1 ? (b[0] >> 4) + ((uint32_t)b[1] << 4)
                                            : (sf == 3 ? (b[0] >> 4) + ((uint32_t)b[1] << 4) + ((uint32_t)b[2] << 12) : (uint32_t)b[0] >> 3);
                            comp = lt == 0 ? regen : 1u;
                        }
                    } else {
                        lh = sf < 2 ? 3 : (sf == 2 ? 4 : 5);
                        if (bsize >= lh) {
                            uint64_t h = 0;
                            for (uint32_t k = 0; k < lh; k++) h |= (uint64_t)b[k] << (8 * k);
                            const uint32_t w = sf < 2 ? 10 : (sf == 2 ? 14 : 18);
                            regen = (uint32_t)((h >> 4) & ((1u << w) - 1u));
                            comp = (uint32_t)((h >> (4 + w)) & ((1u << w) - 1u));
                        }
                    }
                    const uint64_t sec = (uint64_t)lh + comp;
                    if (lh && bsize >= lh && sec < bsize && b[sec] == 0) cb = regen;  // no sequences: the literals
                }
                bound += cb;
            }
            pos += bsize;
        }
        if (bh & 1u) break;
    }
    return bound;
}

// ---------------------------------------------------------------------------------------------
// Backward bit reader (BIT_DStream semantics: the last byte's highest set bit is the end mark;
// bits below position 0 read as zero and flag an overrun).
// ---------------------------------------------------------------------------------------------
struct BitR {
    const uint8_t* s;
    int64_t pos;  // number of unread bits (next bit to read is pos - 1)
};
PGN_HD bool br_init(BitR& b, const uint8_t* src, size_t n)
{
    b.s = src;
    if (n == 0) return false;
    uint8_t last = src[n - 1];
    if (last == 0) return false;
    b.pos = (int64_t)(n - 1) * 8 + (int64_t)highbit32(last);
    return true;
}
// value of the nb bits just below pos (bit pos-1 is the MSB); does not consume
PGN_HD uint32_t br_peek(const BitR& b, unsigned nb)
{
    if (nb == 0) return 0;
    int64_t lo = b.pos - (int64_t)nb;
    uint32_t v = 0;
    int64_t start = lo < 0 ? 0 : lo;
    // gather bits [start, b.pos) -- at most 32 bits
    int64_t byte0 = start >> 3;
    int64_t byte1 = (b.pos - 1) >> 3;
    if (b.pos <= 0) return 0;
    uint64_t acc = 0;
    for (int64_t k = byte1; k >= byte0; k--) acc = (acc << 8) | b.s[k];
    acc >>= (start - (byte0 << 3));
    unsigned width = (unsigned)(b.pos - start);
    v = (uint32_t)(acc & ((width >= 32) ? 0xFFFFFFFFull : ((1ull << width) - 1)));
    if (lo < 0) v <<= (unsigned)(-lo);
    return v;
}
PGN_HD uint32_t br_read(BitR& b, unsigned nb)
{
    uint32_t v = br_peek(b, nb);
    b.pos -= nb;
    return v;
}

// ---------------------------------------------------------------------------------------------
// FSE decoding tables
// ---------------------------------------------------------------------------------------------
struct FseDEntry {
    uint16_t newState;
    uint8_t symbol;
    uint8_t nbBits;
};
struct FseDTable {
    unsigned tableLog;
    FseDEntry e[1 << kLLFSELog];
};

// FSE_readNCount. Returns header bytes consumed, 0 on error.
PGN_HD size_t fse_read_ncount(int16_t* norm, unsigned* maxSVPtr, unsigned* tableLogPtr, const uint8_t* src, size_t srcSize,
                              unsigned maxLogAllowed)
{
    // pad the input to 4 bytes as libzstd does (FSE_readNCount with hbSize < 4)
    uint8_t pad[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint8_t* istart = src;
    size_t hb = srcSize;
    if (hb < 8) {
        for (size_t i = 0; i < hb; i++) pad[i] = src[i];
        istart = pad;
        hb = 8;
    }
    const uint8_t* ip = istart;
    const uint8_t* iend = istart + hb;
    unsigned maxSV1 = *maxSVPtr + 1;
    int previous0 = 0;
    for (unsigned i = 0; i < maxSV1; i++) norm[i] = 0;
    uint32_t bitStream = rd32(ip);
    unsigned nbBits = (bitStream & 0xF) + kFseMinTableLog;
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
                    bitStream = rd32(ip) >> bitCount;
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
                bitStream = rd32(ip) >> bitCount;
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
            bitStream = rd32(ip) >> (bitCount & 31);
        }
    }
    if (remaining != 1) return 0;
    if (bitCount > 32) return 0;
    *maxSVPtr = charnum - 1;
    ip += (bitCount + 7) >> 3;
    size_t used = (size_t)(ip - istart);
    if (used > srcSize) return 0;
    return used;
}

PGN_HD bool fse_build_dtable(FseDTable& dt, const int16_t* norm, unsigned maxSV, unsigned tableLog)
{
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t mask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    uint32_t highThreshold = tableSize - 1;
    uint16_t symbolNext[kMaxML + 1];
    dt.tableLog = tableLog;
    for (unsigned s = 0; s <= maxSV; s++) {
        if (norm[s] == -1) {
            dt.e[highThreshold--].symbol = (uint8_t)s;
            symbolNext[s] = 1;
        } else {
            symbolNext[s] = (uint16_t)norm[s];
        }
    }
    uint32_t position = 0;
    for (unsigned s = 0; s <= maxSV; s++) {
        for (int i = 0; i < norm[s]; i++) {
            dt.e[position].symbol = (uint8_t)s;
            position = (position + step) & mask;
            while (position > highThreshold) position = (position + step) & mask;
        }
    }
    if (position != 0) return false;
    for (uint32_t u = 0; u < tableSize; u++) {
        uint8_t s = dt.e[u].symbol;
        uint32_t nextState = symbolNext[s]++;
        dt.e[u].nbBits = (uint8_t)(tableLog - highbit32(nextState));
        dt.e[u].newState = (uint16_t)((nextState << dt.e[u].nbBits) - tableSize);
    }
    return true;
}
PGN_HD void fse_build_dtable_rle(FseDTable& dt, unsigned symbol)
{
    dt.tableLog = 0;
    dt.e[0].symbol = (uint8_t)symbol;
    dt.e[0].nbBits = 0;
    dt.e[0].newState = 0;
}

// ---------------------------------------------------------------------------------------------
// Huffman decoding (single-symbol table, tableLog <= 12)
// ---------------------------------------------------------------------------------------------
struct HufDEntry {
    uint8_t symbol;
    uint8_t nbBits;
};
struct HufDTable {
    unsigned tableLog;
    HufDEntry e[1 << kHufTableLogMax];
};

// HUF_readStats: the weight list of a Huffman table description (direct 4-bit or FSE-compressed).
// Writes nbW weights (the implied last weight is NOT added).  Returns header bytes consumed, 0 on
// error.
PGN_HD size_t huf_read_weights(uint8_t* weights, unsigned* nbWOut, const uint8_t* src, size_t srcSize, FseDTable& scratchDt)
{
    if (srcSize < 1) return 0;
    unsigned nbW;
    size_t iSize = src[0];
    size_t used;
    if (iSize >= 128) {
        nbW = (unsigned)iSize - 127;
        size_t bytes = (nbW + 1) / 2;
        if (bytes + 1 > srcSize) return 0;
        for (unsigned n = 0; n < nbW; n += 2) {
            weights[n] = src[1 + n / 2] >> 4;
            if (n + 1 < nbW) weights[n + 1] = src[1 + n / 2] & 15;
        }
        used = bytes + 1;
    } else {
        if (iSize + 1 > srcSize) return 0;
        int16_t norm[kHufTableLogMax + 1];
        unsigned maxSV = kHufTableLogMax, tl = 0;
        size_t nc = fse_read_ncount(norm, &maxSV, &tl, src + 1, iSize, 6);
        if (nc == 0 || nc >= iSize) return 0;
        if (!fse_build_dtable(scratchDt, norm, maxSV, tl)) return 0;
        BitR br;
        if (!br_init(br, src + 1 + nc, iSize - nc)) return 0;
        uint32_t st1 = br_read(br, tl), st2 = br_read(br, tl);
        nbW = 0;
        // alternate states; stop when the stream overruns (FSE_decompress_usingDTable tail rule)
        while (true) {
            if (nbW > 253) return 0;
            const FseDEntry e1 = scratchDt.e[st1];
            weights[nbW++] = e1.symbol;
            st1 = e1.newState + br_read(br, e1.nbBits);
            if (br.pos < 0) { weights[nbW++] = scratchDt.e[st2].symbol; break; }
            if (nbW > 253) return 0;
            const FseDEntry e2 = scratchDt.e[st2];
            weights[nbW++] = e2.symbol;
            st2 = e2.newState + br_read(br, e2.nbBits);
            if (br.pos < 0) { weights[nbW++] = scratchDt.e[st1].symbol; break; }
        }
        used = iSize + 1;
    }
    *nbWOut = nbW;
    return used;
}

// The implied last weight and the table log (HUF_readStats tail).  weights[nbW] receives the last
// weight; returns the table log, 0 on error.
PGN_HD unsigned huf_complete_weights(uint8_t* weights, unsigned nbW)
{
    uint32_t rankStats[kHufTableLogMax + 2];
    for (unsigned i = 0; i < kHufTableLogMax + 2; i++) rankStats[i] = 0;
    uint32_t weightTotal = 0;
    for (unsigned n = 0; n < nbW; n++) {
        if (weights[n] > kHufTableLogMax) return 0;
        rankStats[weights[n]]++;
        weightTotal += (1u << weights[n]) >> 1;
    }
    if (weightTotal == 0) return 0;
    unsigned tableLog = highbit32(weightTotal) + 1;
    if (tableLog > kHufTableLogMax) return 0;
    uint32_t total = 1u << tableLog;
    uint32_t rest = total - weightTotal;
    uint32_t verif = 1u << highbit32(rest);
    if (verif != rest) return 0;
    unsigned lastWeight = highbit32(rest) + 1;
    weights[nbW] = (uint8_t)lastWeight;
    rankStats[lastWeight]++;
    if ((rankStats[1] < 2) || (rankStats[1] & 1)) return 0;
    return tableLog;
}

// HUF_readStats + HUF_readDTableX1.  Returns header bytes consumed, 0 on error.
PGN_HD size_t huf_read_dtable(HufDTable& dt, const uint8_t* src, size_t srcSize, FseDTable& scratchDt)
{
    uint8_t weights[256];
    unsigned nbW = 0;
    size_t used = huf_read_weights(weights, &nbW, src, srcSize, scratchDt);
    if (used == 0) return 0;
    unsigned tableLog = huf_complete_weights(weights, nbW);
    if (tableLog == 0) return 0;
    unsigned nbSymbols = nbW + 1;
    uint32_t rankStats[kHufTableLogMax + 2];
    for (unsigned i = 0; i < kHufTableLogMax + 2; i++) rankStats[i] = 0;
    for (unsigned n = 0; n < nbSymbols; n++) rankStats[weights[n]]++;
    // fill the table: weight 1 codes first
    uint32_t rankStart[kHufTableLogMax + 2];
    uint32_t next = 0;
    for (unsigned w = 1; w < tableLog + 1; w++) {
        rankStart[w] = next;
        next += rankStats[w] << (w - 1);
    }
    dt.tableLog = tableLog;
    for (unsigned n = 0; n < nbSymbols; n++) {
        unsigned w = weights[n];
        if (w == 0) continue;
        uint32_t len = (1u << w) >> 1;
        uint32_t u0 = rankStart[w];
        for (uint32_t u = u0; u < u0 + len; u++) {
            dt.e[u].symbol = (uint8_t)n;
            dt.e[u].nbBits = (uint8_t)(tableLog + 1 - w);
        }
        rankStart[w] = u0 + len;
    }
    return used;
}

// Decode one Huffman bitstream of exactly dstSize symbols.  Returns false on corruption.
PGN_HD bool huf_decode_stream(const HufDTable& dt, const uint8_t* src, size_t srcSize, uint8_t* dst, size_t dstSize)
{
    BitR br;
    if (!br_init(br, src, srcSize)) return false;
    const unsigned tl = dt.tableLog;
    for (size_t i = 0; i < dstSize; i++) {
        uint32_t idx = br_peek(br, tl);
        const HufDEntry e = dt.e[idx];
        dst[i] = e.symbol;
        br.pos -= e.nbBits;
    }
    return br.pos == 0;
}

// ---------------------------------------------------------------------------------------------
// Frame decoding state
// ---------------------------------------------------------------------------------------------
struct DecWork {
    HufDTable huf;
    bool hufValid;
    FseDTable ll, of, ml, scratch;
    bool llValid, ofValid, mlValid;
    uint32_t rep[3];
    uint8_t lit[kMaxSrc];  // literal buffer of one block (<= 128 KiB)
};

// Literals section.  Returns bytes consumed (0 on error); *litPtr/*litSize describe the literals
// (either inside src, or in w.lit).
PGN_HD size_t decode_literals(const uint8_t* src, size_t srcSize, DecWork& w, const uint8_t** litPtr, size_t* litSize)
{
    if (srcSize < 1) return 0;
    unsigned type = src[0] & 3, sf = (src[0] >> 2) & 3;
    if (type == kSetBasic || type == kSetRle) {
        size_t lh, rs;
        if (sf == 0 || sf == 2) { lh = 1; rs = src[0] >> 3; }
        else if (sf == 1) { if (srcSize < 2) return 0; lh = 2; rs = (src[0] >> 4) + ((size_t)src[1] << 4); }
        else { if (srcSize < 3) return 0; lh = 3; rs = (src[0] >> 4) + ((size_t)src[1] << 4) + ((size_t)src[2] << 12); }
        if (rs > kMaxSrc) return 0;
        if (type == kSetBasic) {
            if (lh + rs > srcSize) return 0;
            *litPtr = src + lh;
            *litSize = rs;
            return lh + rs;
        }
        if (lh + 1 > srcSize) return 0;
        for (size_t i = 0; i < rs; i++) w.lit[i] = src[lh];
        *litPtr = w.lit;
        *litSize = rs;
        return lh + 1;
    }
    // compressed / treeless
    size_t lh, rs, cs;
    bool single = false;
    if (srcSize < 5) return 0;
    uint32_t lhc = rd32(src);
    if (sf <= 1) { lh = 3; single = (sf == 0); rs = (lhc >> 4) & 0x3FF; cs = (lhc >> 14) & 0x3FF; }
    else if (sf == 2) { lh = 4; rs = (lhc >> 4) & 0x3FFF; cs = lhc >> 18; }
    else { lh = 5; rs = (lhc >> 4) & 0x3FFFF; cs = (lhc >> 22) + ((size_t)src[4] << 10); }
    if (rs > kMaxSrc || lh + cs > srcSize) return 0;
    const uint8_t* ip = src + lh;
    size_t remain = cs;
    if (type == kSetCompressed) {
        size_t h = huf_read_dtable(w.huf, ip, remain, w.scratch);
        if (h == 0) return 0;
        w.hufValid = true;
        ip += h;
        remain -= h;
    } else if (!w.hufValid) {
        return 0;
    }
    if (single) {
        if (!huf_decode_stream(w.huf, ip, remain, w.lit, rs)) return 0;
    } else {
        if (remain < 6) return 0;
        size_t l1 = ip[0] | (ip[1] << 8), l2 = ip[2] | (ip[3] << 8), l3 = ip[4] | (ip[5] << 8);
        if (l1 + l2 + l3 + 6 > remain) return 0;
        size_t l4 = remain - 6 - l1 - l2 - l3;
        size_t seg = (rs + 3) / 4;
        if (seg * 3 > rs) return 0;
        const uint8_t* p = ip + 6;
        if (!huf_decode_stream(w.huf, p, l1, w.lit, seg)) return 0;
        if (!huf_decode_stream(w.huf, p + l1, l2, w.lit + seg, seg)) return 0;
        if (!huf_decode_stream(w.huf, p + l1 + l2, l3, w.lit + 2 * seg, seg)) return 0;
        if (!huf_decode_stream(w.huf, p + l1 + l2 + l3, l4, w.lit + 3 * seg, rs - 3 * seg)) return 0;
    }
    *litPtr = w.lit;
    *litSize = rs;
    return lh + cs;
}

// One sequence table (mode: 0 predefined, 1 rle, 2 fse, 3 repeat).  Returns bytes consumed or
// (size_t)-1 on error.
PGN_HD size_t build_seq_dtable(FseDTable& dt, bool& valid, unsigned mode, const uint8_t* src, size_t srcSize, int kind)
{
    const unsigned maxS = kind == 0 ? kMaxLL : (kind == 1 ? kMaxOff : kMaxML);
    const unsigned maxLog = kind == 0 ? kLLFSELog : (kind == 1 ? kOffFSELog : kMLFSELog);
    int16_t norm[kMaxML + 1];
    if (mode == kSetBasic) {
        unsigned dmax = kind == 0 ? kMaxLL : (kind == 1 ? kDefaultMaxOff : kMaxML);
        for (unsigned s = 0; s <= dmax; s++)
            norm[s] = kind == 0 ? ll_default_norm(s) : (kind == 1 ? of_default_norm(s) : ml_default_norm(s));
        fse_build_dtable(dt, norm, dmax, kind == 0 ? kLLDefaultNormLog : (kind == 1 ? kOFDefaultNormLog : kMLDefaultNormLog));
        valid = true;
        return 0;
    }
    if (mode == kSetRle) {
        if (srcSize < 1 || src[0] > maxS) return (size_t)-1;
        fse_build_dtable_rle(dt, src[0]);
        valid = true;
        return 1;
    }
    if (mode == kSetCompressed) {
        unsigned maxSV = maxS, tl = 0;
        size_t nc = fse_read_ncount(norm, &maxSV, &tl, src, srcSize, maxLog);
        if (nc == 0) return (size_t)-1;
        if (!fse_build_dtable(dt, norm, maxSV, tl)) return (size_t)-1;
        valid = true;
        return nc;
    }
    return valid ? 0 : (size_t)-1;
}

PGN_HD uint32_t of_value(unsigned code, BitR& br)  // offset value per RFC: (1 << code) + bits
{
    return (1u << code) + br_read(br, code);
}

// Sequences section + execution into out (block output starts at out[0]; the window before it
// is out[-winBefore..-1]).  Returns bytes produced or negative error.
PGN_HD long decode_sequences_exec(const uint8_t* src, size_t srcSize, const uint8_t* lit, size_t litSize, DecWork& w,
                                  uint8_t* out, size_t outCap, size_t winBefore)
{
    if (srcSize < 1) return kDecErrCorrupt;
    size_t nbSeq = src[0];
    size_t pos = 1;
    if (nbSeq >= 128) {
        if (nbSeq == 255) {
            if (srcSize < 3) return kDecErrCorrupt;
            nbSeq = (size_t)(src[1] | (src[2] << 8)) + 0x7F00;
            pos = 3;
        } else {
            if (srcSize < 2) return kDecErrCorrupt;
            nbSeq = ((nbSeq - 128) << 8) + src[1];
            pos = 2;
        }
    }
    size_t op = 0;
    if (nbSeq == 0) {
        if (pos != srcSize) return kDecErrCorrupt;
        if (litSize > outCap) return kDecErrDstSmall;
        for (size_t i = 0; i < litSize; i++) out[i] = lit[i];
        return (long)litSize;
    }
    if (pos >= srcSize) return kDecErrCorrupt;
    uint8_t modes = src[pos++];
    size_t r;
    r = build_seq_dtable(w.ll, w.llValid, modes >> 6, src + pos, srcSize - pos, 0);
    if (r == (size_t)-1) return kDecErrCorrupt;
    pos += r;
    r = build_seq_dtable(w.of, w.ofValid, (modes >> 4) & 3, src + pos, srcSize - pos, 1);
    if (r == (size_t)-1) return kDecErrCorrupt;
    pos += r;
    r = build_seq_dtable(w.ml, w.mlValid, (modes >> 2) & 3, src + pos, srcSize - pos, 2);
    if (r == (size_t)-1) return kDecErrCorrupt;
    pos += r;
    BitR br;
    if (!br_init(br, src + pos, srcSize - pos)) return kDecErrCorrupt;
    uint32_t sLL = br_read(br, w.ll.tableLog);
    uint32_t sOF = br_read(br, w.of.tableLog);
    uint32_t sML = br_read(br, w.ml.tableLog);
    size_t litPos = 0;
    for (size_t i = 0; i < nbSeq; i++) {
        const FseDEntry eLL = w.ll.e[sLL], eOF = w.of.e[sOF], eML = w.ml.e[sML];
        unsigned ofCode = eOF.symbol, mlCode = eML.symbol, llCode = eLL.symbol;
        if (ofCode > 31) return kDecErrCorrupt;
        uint32_t ofv = of_value(ofCode, br);
        uint32_t ml = ml_base(mlCode) + br_read(br, ml_bits(mlCode));
        uint32_t ll = ll_base(llCode) + br_read(br, ll_bits(llCode));
        uint32_t offset;
        if (ofv > 3) {
            offset = ofv - 3;
            w.rep[2] = w.rep[1];
            w.rep[1] = w.rep[0];
            w.rep[0] = offset;
        } else {
            unsigned idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // 0..3
            if (idx == 0) {
                offset = w.rep[0];
            } else {
                offset = (idx == 3) ? w.rep[0] - 1 : w.rep[idx];
                if (offset == 0) offset = 1;  // corrupted input: libzstd forces 1
                if (idx != 1) w.rep[2] = w.rep[1];
                w.rep[1] = w.rep[0];
                w.rep[0] = offset;
            }
        }
        if (i + 1 < nbSeq) {
            sLL = eLL.newState + br_read(br, eLL.nbBits);
            sML = eML.newState + br_read(br, eML.nbBits);
            sOF = eOF.newState + br_read(br, eOF.nbBits);
        }
        // execute
        if (litPos + ll > litSize) return kDecErrCorrupt;
        if (op + ll + ml > outCap) return kDecErrDstSmall;
        for (uint32_t k = 0; k < ll; k++) out[op + k] = lit[litPos + k];
        litPos += ll;
        op += ll;
        if ((size_t)offset > op + winBefore) return kDecErrCorrupt;
        for (uint32_t k = 0; k < ml; k++) out[op + k] = out[(long)op + (long)k - (long)offset];
        op += ml;
    }
    if (br.pos != 0) return kDecErrCorrupt;
    size_t rem = litSize - litPos;
    if (op + rem > outCap) return kDecErrDstSmall;
    for (size_t k = 0; k < rem; k++) out[op + k] = lit[litPos + k];
    op += rem;
    return (long)op;
}

// ZSTD_decompress semantics over possibly several concatenated (or skippable) frames.
// Returns decompressed size (>= 0) or a negative DecErr.
PGN_HD long decompress_frames(const uint8_t* src, size_t srcSize, uint8_t* dst, size_t dstCap, DecWork& w)
{
    size_t ip = 0, op = 0;
    if (srcSize == 0) return kDecErrSrcSmall;
    while (ip < srcSize) {
        if (srcSize - ip < 4) return kDecErrSrcSmall;
        uint32_t magic = rd32(src + ip);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (srcSize - ip < 8) return kDecErrSrcSmall;
            uint32_t fs = rd32(src + ip + 4);
            if (fs > srcSize - ip - 8) return kDecErrSrcSmall;
            ip += 8 + fs;
            continue;
        }
        if (magic != kMagic) return kDecErrHeader;
        if (srcSize - ip < 6) return kDecErrSrcSmall;
        uint8_t fhd = src[ip + 4];
        unsigned dictIDFlag = fhd & 3, checksum = (fhd >> 2) & 1, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
        if (fhd & 0x08) return kDecErrHeader;
        size_t hpos = ip + 5;
        uint64_t windowSize = 0;
        if (!singleSegment) {
            uint8_t wd = src[hpos++];
            unsigned exponent = wd >> 3, mantissa = wd & 7;
            uint64_t wb = 1ull << (10 + exponent);
            windowSize = wb + (wb / 8) * mantissa;
        }
        const unsigned didSize[4] = {0, 1, 2, 4};
        uint32_t dictID = 0;
        if (hpos + didSize[dictIDFlag] > srcSize) return kDecErrSrcSmall;
        for (unsigned k = 0; k < didSize[dictIDFlag]; k++) dictID |= (uint32_t)src[hpos + k] << (8 * k);
        hpos += didSize[dictIDFlag];
        if (dictID != 0) return kDecErrHeader;  // no dictionary available
        unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
        if (hpos + fcsSize > srcSize) return kDecErrSrcSmall;
        uint64_t fcs = 0;
        bool hasFcs = fcsSize > 0;
        if (fcsSize == 1) fcs = src[hpos];
        else if (fcsSize == 2) fcs = (uint64_t)(src[hpos] | (src[hpos + 1] << 8)) + 256;
        else if (fcsSize == 4) fcs = rd32(src + hpos);
        else if (fcsSize == 8) fcs = rd64(src + hpos);
        hpos += fcsSize;
        if (singleSegment) windowSize = fcs;
        (void)windowSize;
        ip = hpos;
        size_t frameStart = op;
        w.hufValid = false;
        w.llValid = w.ofValid = w.mlValid = false;
        w.rep[0] = 1; w.rep[1] = 4; w.rep[2] = 8;
        while (true) {
            if (srcSize - ip < 3) return kDecErrSrcSmall;
            uint32_t bh = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8) | ((uint32_t)src[ip + 2] << 16);
            ip += 3;
            unsigned last = bh & 1, btype = (bh >> 1) & 3;
            size_t bsize = bh >> 3;
            if (btype == 3) return kDecErrCorrupt;
            if (btype == kBtRaw) {
                if (bsize > srcSize - ip) return kDecErrSrcSmall;
                if (op + bsize > dstCap) return kDecErrDstSmall;
                for (size_t k = 0; k < bsize; k++) dst[op + k] = src[ip + k];
                ip += bsize;
                op += bsize;
            } else if (btype == kBtRle) {
                if (ip + 1 > srcSize) return kDecErrSrcSmall;
                if (op + bsize > dstCap) return kDecErrDstSmall;
                for (size_t k = 0; k < bsize; k++) dst[op + k] = src[ip];
                ip += 1;
                op += bsize;
            } else {
                if (bsize > srcSize - ip) return kDecErrSrcSmall;
                if (bsize > kMaxSrc) return kDecErrCorrupt;
                const uint8_t* lit;
                size_t litSize;
                size_t lc = decode_literals(src + ip, bsize, w, &lit, &litSize);
                if (lc == 0) return kDecErrCorrupt;
                long r = decode_sequences_exec(src + ip + lc, bsize - lc, lit, litSize, w, dst + op, dstCap - op,
                                               op - frameStart);
                if (r < 0) return r;
                op += (size_t)r;
                ip += bsize;
            }
            if (last) break;
        }
        if (hasFcs && (op - frameStart) != fcs) return kDecErrCorrupt;
        if (checksum) {
            if (srcSize - ip < 4) return kDecErrSrcSmall;
            ip += 4;  // XXH64 low 32 bits: not verified
        }
    }
    return (long)op;
}

}  // namespace z1
}  // namespace pgn
