// pgn_zdec.h -- one wave decodes the zstd frame(s) of one stream (ZSTD_decompress semantics, the
// call at C5.hpp:588-667).  Headers, Huffman/FSE table builds and the sequence list run on lane 0
// with the shared zstd1_dec.h code; raw/RLE blocks, literal copies and match copies use the whole
// wave; the (up to four) Huffman streams of a literals section are decoded one per lane.
#pragma once
#include "pgn_wave.h"
#include "zstd1_dec.h"

namespace pgn {

struct DecLds {
    z1::HufDTable huf;     // 8 KiB
    z1::FseDTable fscr;    // weights table scratch
    uint32_t u[16];
};

struct DecScratch {
    uint8_t* lit;           // literals of a block with sequences (<= 128 KiB)
    uint32_t* seqs;         // decoded sequences: {litLength, matchLength, offset} triples
    uint32_t maxSeq;
    z1::FseDTable* tables;  // ll, of, ml
};

// Backward bit reader with a 64-bit window, for the per-lane Huffman streams.
struct BitWin {
    const uint8_t* s;
    int64_t pos;  // unread bits
    int64_t wlo;  // w holds bits [wlo, wlo + 64)
    uint64_t w;
};
__device__ __forceinline__ void bw_refill(BitWin& b)
{
    int64_t byteEnd = (b.pos + 7) >> 3;
    int64_t byteLo = byteEnd - 8;
    if (byteLo >= 0) {
        b.w = ld64u(b.s + byteLo);
    } else {
        byteLo = 0;
        uint64_t v = 0;
        for (int64_t k = byteEnd - 1; k >= 0; k--) v = (v << 8) | b.s[k];
        b.w = v;
    }
    b.wlo = byteLo * 8;
}
__device__ __forceinline__ uint32_t bw_peek(const BitWin& b, unsigned nb)
{
    int64_t lo = b.pos - (int64_t)nb;
    uint64_t m = (1ull << nb) - 1;
    if (lo >= b.wlo) return (uint32_t)((b.w >> (lo - b.wlo)) & m);
    return (uint32_t)((b.w << (b.wlo - lo)) & m);  // only at the stream start (wlo == 0)
}

__device__ inline bool huf_decode_stream_lane(const z1::HufDTable& dt, const uint8_t* src, size_t srcSize, uint8_t* dst,
                                              size_t dstSize)
{
    if (srcSize == 0) return false;
    const uint8_t last = src[srcSize - 1];
    if (last == 0) return false;
    BitWin b;
    b.s = src;
    b.pos = (int64_t)(srcSize - 1) * 8 + (int64_t)z1::highbit32(last);
    bw_refill(b);
    const unsigned tl = dt.tableLog;
    for (size_t i = 0; i < dstSize; i++) {
        if (b.pos - b.wlo < (int64_t)tl && b.wlo > 0) bw_refill(b);
        const z1::HufDEntry e = dt.e[bw_peek(b, tl)];
        dst[i] = e.symbol;
        b.pos -= e.nbBits;
    }
    return b.pos == 0;
}

// Decode the sequences section into a list (lane 0).  Returns nbSeq or -1.
__device__ inline long decode_seq_list(const uint8_t* src, size_t srcSize, const DecScratch& S, uint32_t rep[3],
                                       bool valid[3])
{
    size_t nbSeq = src[0];
    size_t pos = 1;
    if (nbSeq >= 128) {
        if (nbSeq == 255) {
            if (srcSize < 3) return -1;
            nbSeq = (size_t)(src[1] | (src[2] << 8)) + 0x7F00;
            pos = 3;
        } else {
            if (srcSize < 2) return -1;
            nbSeq = ((nbSeq - 128) << 8) + src[1];
            pos = 2;
        }
    }
    if (nbSeq == 0) return (pos == srcSize) ? 0 : -1;
    if (nbSeq > S.maxSeq || pos >= srcSize) return -1;
    const uint8_t modes = src[pos++];
    z1::FseDTable& ll = S.tables[0];
    z1::FseDTable& of = S.tables[1];
    z1::FseDTable& ml = S.tables[2];
    size_t r = z1::build_seq_dtable(ll, valid[0], modes >> 6, src + pos, srcSize - pos, 0);
    if (r == (size_t)-1) return -1;
    pos += r;
    r = z1::build_seq_dtable(of, valid[1], (modes >> 4) & 3, src + pos, srcSize - pos, 1);
    if (r == (size_t)-1) return -1;
    pos += r;
    r = z1::build_seq_dtable(ml, valid[2], (modes >> 2) & 3, src + pos, srcSize - pos, 2);
    if (r == (size_t)-1) return -1;
    pos += r;
    z1::BitR br;
    if (!z1::br_init(br, src + pos, srcSize - pos)) return -1;
    uint32_t sLL = z1::br_read(br, ll.tableLog);
    uint32_t sOF = z1::br_read(br, of.tableLog);
    uint32_t sML = z1::br_read(br, ml.tableLog);
    for (size_t i = 0; i < nbSeq; i++) {
        const z1::FseDEntry eLL = ll.e[sLL], eOF = of.e[sOF], eML = ml.e[sML];
        const unsigned ofCode = eOF.symbol, mlCode = eML.symbol, llCode = eLL.symbol;
        if (ofCode > 31) return -1;
        const uint32_t ofv = z1::of_value(ofCode, br);
        const uint32_t mlen = z1::ml_base(mlCode) + z1::br_read(br, z1::ml_bits(mlCode));
        const uint32_t llen = z1::ll_base(llCode) + z1::br_read(br, z1::ll_bits(llCode));
        uint32_t offset;
        if (ofv > 3) {
            offset = ofv - 3;
            rep[2] = rep[1]; rep[1] = rep[0]; rep[0] = offset;
        } else {
            unsigned idx = ofv - 1 + (llen == 0 ? 1u : 0u);
            if (idx == 0) {
                offset = rep[0];
            } else {
                offset = (idx == 3) ? rep[0] - 1 : rep[idx];
                if (offset == 0) offset = 1;
                if (idx != 1) rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = offset;
            }
        }
        if (i + 1 < nbSeq) {
            sLL = eLL.newState + z1::br_read(br, eLL.nbBits);
            sML = eML.newState + z1::br_read(br, eML.nbBits);
            sOF = eOF.newState + z1::br_read(br, eOF.nbBits);
        }
        S.seqs[3 * i] = llen;
        S.seqs[3 * i + 1] = mlen;
        S.seqs[3 * i + 2] = offset;
    }
    if (br.pos != 0) return -1;
    return (long)nbSeq;
}

// ZSTD_decompress(dst, dstCap, src, srcSize).  Returns size or a negative z1::DecErr.
__device__ inline long zstd_decompress_wave(const uint8_t* __restrict__ src, size_t srcSize, uint8_t* __restrict__ dst,
                                            size_t dstCap, DecLds& L, const DecScratch& S)
{
    const int lane = lane_id();
    size_t ip = 0, op = 0;
    if (srcSize == 0) return z1::kDecErrSrcSmall;
    while (ip < srcSize) {
        if (srcSize - ip < 4) return z1::kDecErrSrcSmall;
        const uint32_t magic = ld32u(src + ip);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (srcSize - ip < 8) return z1::kDecErrSrcSmall;
            uint32_t fs = ld32u(src + ip + 4);
            if (fs > srcSize - ip - 8) return z1::kDecErrSrcSmall;
            ip += 8 + (size_t)fs;
            continue;
        }
        if (magic != z1::kMagic) return z1::kDecErrHeader;
        if (srcSize - ip < 6) return z1::kDecErrSrcSmall;
        const uint8_t fhd = src[ip + 4];
        const unsigned dictIDFlag = fhd & 3, checksum = (fhd >> 2) & 1, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
        if (fhd & 0x08) return z1::kDecErrHeader;
        size_t hpos = ip + 5 + (singleSegment ? 0 : 1);
        const unsigned didSize = dictIDFlag == 0 ? 0 : (dictIDFlag == 1 ? 1 : (dictIDFlag == 2 ? 2 : 4));
        if (hpos + didSize > srcSize) return z1::kDecErrSrcSmall;
        uint32_t dictID = 0;
        for (unsigned k = 0; k < didSize; k++) dictID |= (uint32_t)src[hpos + k] << (8 * k);
        hpos += didSize;
        if (dictID != 0) return z1::kDecErrHeader;
        const unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
        if (hpos + fcsSize > srcSize) return z1::kDecErrSrcSmall;
        uint64_t fcs = 0;
        if (fcsSize == 1) fcs = src[hpos];
        else if (fcsSize == 2) fcs = (uint64_t)(src[hpos] | (src[hpos + 1] << 8)) + 256;
        else if (fcsSize == 4) fcs = ld32u(src + hpos);
        else if (fcsSize == 8) fcs = ld64u(src + hpos);
        hpos += fcsSize;
        ip = hpos;
        const size_t frameStart = op;
        bool hufValid = false;
        bool tvalid[3] = {false, false, false};
        uint32_t rep[3] = {1, 4, 8};
        while (true) {
            if (srcSize - ip < 3) return z1::kDecErrSrcSmall;
            const uint32_t bh = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8) | ((uint32_t)src[ip + 2] << 16);
            ip += 3;
            const unsigned last = bh & 1, btype = (bh >> 1) & 3;
            const size_t bsize = bh >> 3;
            if (btype == 3) return z1::kDecErrCorrupt;
            if (btype == z1::kBtRaw) {
                if (bsize > srcSize - ip) return z1::kDecErrSrcSmall;
                if (op + bsize > dstCap) return z1::kDecErrDstSmall;
                wave_copy(dst + op, src + ip, bsize);
                ip += bsize;
                op += bsize;
            } else if (btype == z1::kBtRle) {
                if (ip + 1 > srcSize) return z1::kDecErrSrcSmall;
                if (op + bsize > dstCap) return z1::kDecErrDstSmall;
                wave_fill(dst + op, src[ip], bsize);
                ip += 1;
                op += bsize;
            } else {
                if (bsize > srcSize - ip) return z1::kDecErrSrcSmall;
                if (bsize > z1::kMaxSrc) return z1::kDecErrCorrupt;
                const uint8_t* blk = src + ip;
                // ---- literals section header
                if (bsize < 1) return z1::kDecErrCorrupt;
                const unsigned ltype = blk[0] & 3, sf = (blk[0] >> 2) & 3;
                size_t lh, rs, cs = 0;
                bool single = false;
                if (ltype == z1::kSetBasic || ltype == z1::kSetRle) {
                    if (sf == 0 || sf == 2) { lh = 1; rs = blk[0] >> 3; }
                    else if (sf == 1) { if (bsize < 2) return z1::kDecErrCorrupt; lh = 2; rs = (blk[0] >> 4) + ((size_t)blk[1] << 4); }
                    else { if (bsize < 3) return z1::kDecErrCorrupt; lh = 3; rs = (blk[0] >> 4) + ((size_t)blk[1] << 4) + ((size_t)blk[2] << 12); }
                    cs = (ltype == z1::kSetBasic) ? rs : 1;
                } else {
                    if (bsize < 5) return z1::kDecErrCorrupt;
                    const uint32_t lhc = ld32u(blk);
                    if (sf <= 1) { lh = 3; single = (sf == 0); rs = (lhc >> 4) & 0x3FF; cs = (lhc >> 14) & 0x3FF; }
                    else if (sf == 2) { lh = 4; rs = (lhc >> 4) & 0x3FFF; cs = lhc >> 18; }
                    else { lh = 5; rs = (lhc >> 4) & 0x3FFFF; cs = (lhc >> 22) + ((size_t)blk[4] << 10); }
                }
                if (rs > z1::kMaxSrc || lh + cs > bsize) return z1::kDecErrCorrupt;
                const uint8_t* seqSrc = blk + lh + cs;
                const size_t seqSize = bsize - lh - cs;
                if (seqSize < 1) return z1::kDecErrCorrupt;
                const bool noSeq = (seqSrc[0] == 0);
                if (noSeq && seqSize != 1) return z1::kDecErrCorrupt;
                if (noSeq && op + rs > dstCap) return z1::kDecErrDstSmall;
                uint8_t* litOut = noSeq ? dst + op : S.lit;
                const uint8_t* lit = litOut;
                if (ltype == z1::kSetBasic) {
                    if (noSeq) wave_copy(litOut, blk + lh, rs);
                    else lit = blk + lh;
                } else if (ltype == z1::kSetRle) {
                    wave_fill(litOut, blk[lh], rs);
                } else {
                    const uint8_t* hp = blk + lh;
                    size_t remain = cs;
                    if (ltype == z1::kSetCompressed) {
                        if (lane == 0) L.u[0] = (uint32_t)z1::huf_read_dtable(L.huf, hp, remain, L.fscr);
                        wave_sync();
                        const size_t hsz = L.u[0];
                        if (hsz == 0) return z1::kDecErrCorrupt;
                        hufValid = true;
                        hp += hsz;
                        remain -= hsz;
                    } else if (!hufValid) {
                        return z1::kDecErrCorrupt;
                    }
                    bool ok = true;
                    if (single) {
                        if (lane == 0) ok = huf_decode_stream_lane(L.huf, hp, remain, litOut, rs);
                    } else {
                        if (remain < 6) return z1::kDecErrCorrupt;
                        const size_t l1 = hp[0] | (hp[1] << 8), l2 = hp[2] | (hp[3] << 8), l3 = hp[4] | (hp[5] << 8);
                        if (l1 + l2 + l3 + 6 > remain) return z1::kDecErrCorrupt;
                        const size_t l4 = remain - 6 - l1 - l2 - l3;
                        const size_t seg = (rs + 3) / 4;
                        if (seg * 3 > rs) return z1::kDecErrCorrupt;
                        if (lane < 4) {
                            const size_t so = (lane == 0) ? 0 : (lane == 1 ? l1 : (lane == 2 ? l1 + l2 : l1 + l2 + l3));
                            const size_t sl = (lane == 0) ? l1 : (lane == 1 ? l2 : (lane == 2 ? l3 : l4));
                            const size_t dn = (lane == 3) ? rs - 3 * seg : seg;
                            ok = huf_decode_stream_lane(L.huf, hp + 6 + so, sl, litOut + seg * (size_t)lane, dn);
                        }
                    }
                    if (ballot(!ok)) return z1::kDecErrCorrupt;
                }
                wave_sync();
                if (noSeq) {
                    op += rs;
                } else {
                    // ---- sequences: list on lane 0, execution on the wave
                    if (lane == 0) {
                        long nb = decode_seq_list(seqSrc, seqSize, S, rep, tvalid);
                        L.u[1] = (uint32_t)(nb < 0 ? 0xFFFFFFFFu : (uint32_t)nb);
                        L.u[2] = rep[0]; L.u[3] = rep[1]; L.u[4] = rep[2];
                        L.u[5] = tvalid[0]; L.u[6] = tvalid[1]; L.u[7] = tvalid[2];
                    }
                    wave_sync();
                    const uint32_t nb = L.u[1];
                    if (nb == 0xFFFFFFFFu) return z1::kDecErrCorrupt;
                    rep[0] = L.u[2]; rep[1] = L.u[3]; rep[2] = L.u[4];
                    tvalid[0] = L.u[5]; tvalid[1] = L.u[6]; tvalid[2] = L.u[7];
                    size_t litPos = 0;
                    for (uint32_t i = 0; i < nb; i++) {
                        const uint32_t ll = S.seqs[3 * i], ml = S.seqs[3 * i + 1], off = S.seqs[3 * i + 2];
                        if (litPos + ll > rs) return z1::kDecErrCorrupt;
                        if (op + ll + ml > dstCap) return z1::kDecErrDstSmall;
                        wave_copy(dst + op, lit + litPos, ll);
                        litPos += ll;
                        op += ll;
                        if ((size_t)off > op - frameStart) return z1::kDecErrCorrupt;
                        wave_sync();
                        for (uint32_t k = (uint32_t)lane; k < ml; k += 64) dst[op + k] = dst[op - off + (k % off)];
                        op += ml;
                        wave_sync();
                    }
                    const size_t remLit = rs - litPos;
                    if (op + remLit > dstCap) return z1::kDecErrDstSmall;
                    wave_copy(dst + op, lit + litPos, remLit);
                    op += remLit;
                    wave_sync();
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

}  // namespace pgn
