// pgn_zdec.h -- one wave decodes the zstd frame(s) of one stream (ZSTD_decompress semantics, the
// call at C5.hpp:588-667).  Headers, Huffman/FSE table builds and the sequence list run on lane 0
// with the shared zstd1_dec.h code; raw/RLE blocks, literal copies and match copies use the whole
// wave; the (up to four) Huffman streams of a literals section are decoded one per lane.
#pragma once
#include "pgn_wave.h"
#include "zstd1_dec.h"

namespace pgn {

constexpr int kRec = 16;          // boundary positions recorded per lane for the synchronisation check
constexpr int kStgBytes = 144;    // per-lane LDS staging of compressed bits per round (128 + lookahead)
constexpr int32_t kRoundBits = 1024;

struct DecLds {
    uint16_t tab[1 << z1::kHufTableLogMax];  // Huffman decode table: symbol | nbBits << 8
    uint32_t stg[64][kStgBytes / 4];         // per-lane staged stream bytes of the current round
    uint32_t rec[64][kRec];                  // speculative decode: first boundaries per lane
    uint32_t cnt[64], startp[64], endp[64], exitp[64], tstart[64], tcount[64];
    uint8_t wts[256];                        // weights of the current table
    uint8_t order[256];                      // symbols sorted by (weight, symbol)
    z1::FseDTable fscr;                      // weights FSE table scratch
    uint32_t u[16];
};

// One instance per decode workgroup (namespace scope, so every access is a DS instruction).
static __shared__ DecLds sDec;

struct DecScratch {
    uint8_t* lit;           // literals of a block with sequences (<= 128 KiB)
    uint32_t* seqs;         // decoded sequences: {litLength, matchLength, offset} triples
    uint32_t maxSeq;
    z1::FseDTable* tables;  // ll, of, ml
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
__device__ __forceinline__ uint32_t rb_huf(RevBits& r, int32_t& pos, unsigned tl)
{
    if (pos - r.wlo < (int32_t)tl && r.wlo > 0) rb_fill(r, pos);
    const uint32_t e = sDec.tab[rb_peek(r, pos, tl)];
    pos -= (int32_t)(e >> 8);
    return e & 0xFF;
}

// ---------------------------------------------------------------------------------------------
// Round-staged reader: lane l's stream bytes [base, base + kStgBytes) live in sDec.stg[l]; stage
// positions are bit offsets from base*8.  W caches 64 bits at stage word index wi.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void stage_round(const uint8_t* __restrict__ src, int32_t roundHi, int lane, int32_t& base)
{
    const int32_t byteHi = (roundHi + 7) >> 3;
    base = byteHi - kStgBytes;
    uint32_t* d = sDec.stg[lane];
    if (base >= 0) {
        uint4 v[kStgBytes / 16];
#pragma unroll
        for (int q = 0; q < kStgBytes / 16; q++) v[q] = gld<uint4>(src + base + 16 * q);
#pragma unroll
        for (int q = 0; q < kStgBytes / 16; q++) {
            d[4 * q] = v[q].x; d[4 * q + 1] = v[q].y; d[4 * q + 2] = v[q].z; d[4 * q + 3] = v[q].w;
        }
    } else {  // the first bytes of the stream: zero below byte 0
        for (int q = 0; q < kStgBytes / 4; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int32_t idx = base + 4 * q + b;
                if (idx >= 0 && idx < byteHi) v |= (uint32_t)gb(src + idx) << (8 * b);
            }
            d[q] = v;
        }
    }
}
struct StgBits {
    uint64_t W;   // stage bits [32*wi, 32*wi + 64)
    int32_t wi;   // word index of W's low word
};
__device__ __forceinline__ void sb_fill(StgBits& r, int lane, int32_t q)  // q: stage bit position
{
    int32_t wi = (q >> 5) - 1;
    wi = wi < 0 ? 0 : wi;
    r.wi = wi;
    r.W = (uint64_t)sDec.stg[lane][wi] | ((uint64_t)sDec.stg[lane][wi + 1] << 32);
}
// decode one symbol whose code ends at stage bit q (bits [q - tl, q)); returns the table entry
__device__ __forceinline__ uint32_t sb_huf(StgBits& r, int lane, int32_t q, unsigned tl)
{
    if (q - (int32_t)tl < 32 * r.wi || q > 32 * r.wi + 64) sb_fill(r, lane, q);
    const int32_t lo = q - (int32_t)tl;
    const uint32_t idx = (lo >= 32 * r.wi) ? (uint32_t)(r.W >> (lo - 32 * r.wi)) : (uint32_t)(r.W << (32 * r.wi - lo));
    return sDec.tab[idx & ((1u << tl) - 1)];
}

// ---------------------------------------------------------------------------------------------
// Huffman table description -> decode table in LDS (HUF_readStats + HUF_readDTableX1).  The weight
// list is parsed on lane 0; ranking and the table fill use the whole wave.  Returns header bytes
// consumed (0 = corrupt); *tlOut = table log.
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ size_t huf_build_dtable_wave(const uint8_t* src, size_t srcSize, unsigned* tlOut)
{
    const int lane = lane_id();
    src = uni(src);
    srcSize = uni((uint64_t)srcSize);
    if (lane == 0) {
        unsigned nbW = 0;
        size_t used = z1::huf_read_weights(sDec.wts, &nbW, src, srcSize, sDec.fscr);
        unsigned tl = used ? z1::huf_complete_weights(sDec.wts, nbW) : 0;
        sDec.u[8] = (uint32_t)used;
        sDec.u[9] = tl;
        sDec.u[10] = nbW + 1;
    }
    lds_sync();
    const size_t used = sDec.u[8];
    const unsigned tl = sDec.u[9];
    const unsigned nbSym = sDec.u[10];
    if (used == 0 || tl == 0) return 0;
    // per-weight counts and exclusive ranks of my four symbols (weights 1..12, 10 bits each)
    uint32_t w4[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t sym = 4u * (uint32_t)lane + (uint32_t)q;
        w4[q] = (sym < nbSym) ? sDec.wts[sym] : 0u;
    }
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
        if (w4[q]) sDec.order[before[w4[q]] + rankIdx[q]] = (uint8_t)sym;
    }
    lds_sync();
    const uint32_t tsize = 1u << tl;
    for (uint32_t u = (uint32_t)lane; u < tsize; u += 64) {
        unsigned w = 1;
#pragma unroll
        for (unsigned ww = 2; ww <= 12; ww++)
            if (ww <= tl && cntW[ww] && u >= rankStart[ww]) w = ww;
        const uint32_t k = (u - rankStart[w]) >> (w - 1);
        sDec.tab[u] = (uint16_t)(sDec.order[before[w] + k] | ((tl + 1 - w) << 8));
    }
    lds_sync();
    *tlOut = tl;
    return used;
}

// ---------------------------------------------------------------------------------------------
// Four Huffman streams decoded by the whole wave: 16 lanes per stream.  Each lane decodes a bit
// range of its stream starting at an assumed codeword boundary (phase 1) and records its first
// boundaries; one lane per stream then chains the true starts: a lane whose recorded boundaries
// contain the previous lane's exit has self-synchronised, otherwise that range is re-decoded serially
// (phase 2); finally every lane decodes its exact symbols from its true start into place (phase 3).
// Compressed bits are staged per lane in LDS, one 1024-bit round at a time, so the inner loops only
// touch LDS and the output stores never stall them.  Returns false on a malformed stream.
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ bool huf_decode4_wave(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs)
{
    const int lane = lane_id();
    tl = uni(tl);
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    dst = uni(dst);
    rs = uni(rs);
    const int k = lane >> 4, j = lane & 15;
    if (remain < 6) return false;
    const size_t l1 = gld<uint16_t>(hp), l2 = gld<uint16_t>(hp + 2), l3 = gld<uint16_t>(hp + 4);
    if (l1 + l2 + l3 + 6 > remain) return false;
    const size_t l4 = remain - 6 - l1 - l2 - l3;
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs) return false;
    const size_t so = (k == 0) ? 0 : (k == 1 ? l1 : (k == 2 ? l1 + l2 : l1 + l2 + l3));
    const size_t sl = (k == 0) ? l1 : (k == 1 ? l2 : (k == 2 ? l3 : l4));
    const uint32_t nsym = (k == 3) ? rs - 3 * seg : seg;
    const uint8_t* src = hp + 6 + so;
    const uint8_t lastB = sl > 0 ? gb(src + sl - 1) : 0;
    if (ballot(lastB == 0)) return false;
    const int32_t B = (int32_t)(sl - 1) * 8 + (int32_t)z1::highbit32(lastB);
    const int32_t Lr = (B + 15) >> 4;
    const int32_t S = (B > j * Lr) ? B - j * Lr : 0;
    const int32_t E = (B > (j + 1) * Lr) ? B - (j + 1) * Lr : 0;

    // ---- phase 1: speculative decode of (E, S], counting symbols, recording the first boundaries
    int32_t pos = S;
    uint32_t c = 0;
    {
        const int32_t rounds = (int32_t)wave_max((uint32_t)((S - E + kRoundBits - 1) / kRoundBits));
        for (int32_t r = 0; r < rounds; r++) {
            const int32_t hi = S - r * kRoundBits;
            const int32_t lo = (hi - kRoundBits > E) ? hi - kRoundBits : E;
            int32_t base = 0;
            if (hi > E) stage_round(src, pos, lane, base);
            lds_sync();
            if (hi > E) {
                StgBits sb;
                sb_fill(sb, lane, pos - 8 * base);
                while (pos > lo) {
                    if (c < (uint32_t)kRec) sDec.rec[lane][c] = (uint32_t)pos;
                    const uint32_t e = sb_huf(sb, lane, pos - 8 * base, tl);
                    pos -= (int32_t)(e >> 8);
                    c++;
                }
            }
            lds_sync();
        }
    }
    sDec.cnt[lane] = c;
    sDec.startp[lane] = (uint32_t)S;
    sDec.endp[lane] = (uint32_t)E;
    sDec.exitp[lane] = (uint32_t)pos;
    lds_sync();
    // ---- phase 2: chain the true starts (one lane per stream)
    if (j == 0) {
        sDec.tstart[lane] = (uint32_t)S;
        sDec.tcount[lane] = c;
        int32_t T = pos;
        RevBits r2;
        r2.s = src;
        for (int jj = 1; jj < 16; jj++) {
            const int l = lane + jj;
            const uint32_t cl = sDec.cnt[l];
            const uint32_t m = cl < (uint32_t)kRec ? cl : (uint32_t)kRec;
            const int32_t El = (int32_t)sDec.endp[l];
            sDec.tstart[l] = (uint32_t)T;
            // walk the true path from T until it meets a boundary the speculative decode recorded
            int32_t p = T;
            uint32_t extra = 0, idx = 0;
            bool synced = false;
            rb_fill(r2, p);
            while (p > El) {
                while (idx < m && (int32_t)sDec.rec[l][idx] > p) idx++;
                if (idx < m && (int32_t)sDec.rec[l][idx] == p) { synced = true; break; }
                if (idx >= m) break;  // past the recorded boundaries: finish serially below
                rb_huf(r2, p, tl);
                extra++;
            }
            if (synced) {
                sDec.tcount[l] = extra + (cl - idx);
                T = (int32_t)sDec.exitp[l];
            } else {
                while (p > El) { rb_huf(r2, p, tl); extra++; }
                sDec.tcount[l] = extra;
                T = p;
            }
        }
        sDec.u[12 + k] = (uint32_t)T;  // true end of the stream (must be 0)
    }
    lds_sync();
    // ---- phase 3: exact decode into place
    const uint32_t tc = sDec.tcount[lane];
    const uint32_t incl = wave_incl_sum(tc);
    // per-lane source lanes: __shfl (ds_bpermute), not readlane (which needs a uniform index)
    const uint32_t grpEnd = (uint32_t)__shfl((int)incl, 16 * k + 15, 64);
    const uint32_t grpBase = (uint32_t)__shfl((int)incl, (16 * k + 63) & 63, 64);
    const uint32_t grpStart = (k == 0) ? 0u : grpBase;
    const bool good = (grpEnd - grpStart == nsym) && ((int32_t)sDec.u[12 + k] == 0);
    if (ballot(!good)) return false;
    uint8_t* out = dst + (size_t)seg * (size_t)k + (incl - tc - grpStart);
    const int32_t T0 = (int32_t)sDec.tstart[lane];
    pos = T0;
    uint32_t i = 0, acc = 0;
    {
        // rounds over this lane's true range, until tc symbols are out
        const int32_t Tend = pos - 0;  // range upper end
        (void)Tend;
        const int32_t span = (int32_t)wave_max((uint32_t)(T0 - (j == 15 ? 0 : (int32_t)sDec.tstart[(lane + 1) & 63])));
        const int32_t rounds = (span + kRoundBits - 1) / kRoundBits + 1;
        for (int32_t r = 0; r < rounds; r++) {
            const bool act = i < tc;
            int32_t base = 0;
            if (act) stage_round(src, pos, lane, base);
            lds_sync();
            if (act) {
                StgBits sb;
                sb_fill(sb, lane, pos - 8 * base);
                const int32_t lo = pos - kRoundBits;
                while (i < tc && pos > lo) {
                    const uint32_t e = sb_huf(sb, lane, pos - 8 * base, tl);
                    pos -= (int32_t)(e >> 8);
                    acc |= (e & 0xFF) << (8 * (i & 3));
                    i++;
                    if ((i & 3) == 0) {
                        gst<uint32_t>(out + i - 4, acc);
                        acc = 0;
                    }
                }
            }
            lds_sync();
        }
        for (uint32_t t = i & ~3u; t < i; t++) gst<uint8_t>(out + t, (uint8_t)(acc >> (8 * (t & 3))));
    }
    return true;
}

// single-stream literals (< 256 symbols in zstd's encoder): lane 0
__device__ __noinline__ bool huf_decode1_lane(unsigned tl, const uint8_t* src, size_t sl, uint8_t* dst, uint32_t n)
{
    if (sl == 0 || gb(src + sl - 1) == 0) return false;
    int32_t pos = (int32_t)(sl - 1) * 8 + (int32_t)z1::highbit32(gb(src + sl - 1));
    RevBits rb;
    rb.s = src;
    rb_fill(rb, pos);
    for (uint32_t i = 0; i < n; i++) gst<uint8_t>(dst + i, (uint8_t)rb_huf(rb, pos, tl));
    return pos == 0;
}

// Decode the sequences section into a list (lane 0).  Returns nbSeq or -1.
__device__ __noinline__ long decode_seq_list(const uint8_t* src, size_t srcSize, const DecScratch& S, uint32_t rep[3],
                                       bool valid[3])
{
    size_t nbSeq = gb(src + (0));
    size_t pos = 1;
    if (nbSeq >= 128) {
        if (nbSeq == 255) {
            if (srcSize < 3) return -1;
            nbSeq = (size_t)(gb(src + (1)) | (gb(src + (2)) << 8)) + 0x7F00;
            pos = 3;
        } else {
            if (srcSize < 2) return -1;
            nbSeq = ((nbSeq - 128) << 8) + gb(src + (1));
            pos = 2;
        }
    }
    if (nbSeq == 0) return (pos == srcSize) ? 0 : -1;
    if (nbSeq > S.maxSeq || pos >= srcSize) return -1;
    const uint8_t modes = gb(src + (pos++));
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

// Sequences of one block: the list on lane 0, execution (literal + match copies) on the wave.
// Returns the new output position or a negative z1::DecErr.
__device__ __noinline__ long exec_sequences_wave(const uint8_t* seqSrc, size_t seqSize, const uint8_t* lit, size_t rs,
                                                 uint8_t* dst, size_t op, size_t dstCap, size_t frameStart,
                                                 DecScratch S, uint32_t rep[3], bool tvalid[3])
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
    S.lit = uni(S.lit);
    S.seqs = uni(S.seqs);
    S.maxSeq = uni(S.maxSeq);
    S.tables = uni(S.tables);
    if (lane == 0) {
        long nb = decode_seq_list(seqSrc, seqSize, S, rep, tvalid);
        sDec.u[1] = (uint32_t)(nb < 0 ? 0xFFFFFFFFu : (uint32_t)nb);
        sDec.u[2] = rep[0]; sDec.u[3] = rep[1]; sDec.u[4] = rep[2];
        sDec.u[5] = tvalid[0]; sDec.u[6] = tvalid[1]; sDec.u[7] = tvalid[2];
    }
    wave_sync();
    const uint32_t nb = sDec.u[1];
    if (nb == 0xFFFFFFFFu) return z1::kDecErrCorrupt;
    rep[0] = sDec.u[2]; rep[1] = sDec.u[3]; rep[2] = sDec.u[4];
    tvalid[0] = sDec.u[5]; tvalid[1] = sDec.u[6]; tvalid[2] = sDec.u[7];
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
        for (uint32_t k = (uint32_t)lane; k < ml; k += 64) gst<uint8_t>(dst + op + k, gb(dst + op - off + (k % off)));
        op += ml;
        wave_sync();
    }
    const size_t remLit = rs - litPos;
    if (op + remLit > dstCap) return z1::kDecErrDstSmall;
    wave_copy(dst + op, lit + litPos, remLit);
    op += remLit;
    wave_sync();
    return (long)op;
}

// ZSTD_decompress(dst, dstCap, src, srcSize).  Returns size or a negative z1::DecErr.
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
        const uint8_t fhd = gb(src + (ip + 4));
        const unsigned dictIDFlag = fhd & 3, checksum = (fhd >> 2) & 1, singleSegment = (fhd >> 5) & 1, fcsFlag = fhd >> 6;
        if (fhd & 0x08) return z1::kDecErrHeader;
        size_t hpos = ip + 5 + (singleSegment ? 0 : 1);
        const unsigned didSize = dictIDFlag == 0 ? 0 : (dictIDFlag == 1 ? 1 : (dictIDFlag == 2 ? 2 : 4));
        if (hpos + didSize > srcSize) return z1::kDecErrSrcSmall;
        uint32_t dictID = 0;
        for (unsigned k = 0; k < didSize; k++) dictID |= (uint32_t)gb(src + (hpos + k)) << (8 * k);
        hpos += didSize;
        if (dictID != 0) return z1::kDecErrHeader;
        const unsigned fcsSize = (fcsFlag == 0) ? (singleSegment ? 1 : 0) : (1u << fcsFlag);
        if (hpos + fcsSize > srcSize) return z1::kDecErrSrcSmall;
        uint64_t fcs = 0;
        if (fcsSize == 1) fcs = gb(src + (hpos));
        else if (fcsSize == 2) fcs = (uint64_t)(gb(src + (hpos)) | (gb(src + (hpos + 1)) << 8)) + 256;
        else if (fcsSize == 4) fcs = ld32u(src + hpos);
        else if (fcsSize == 8) fcs = ld64u(src + hpos);
        hpos += fcsSize;
        ip = hpos;
        const size_t frameStart = op;
        bool hufValid = false;
        unsigned hufTl = 0;
        bool tvalid[3] = {false, false, false};
        uint32_t rep[3] = {1, 4, 8};
        while (true) {
            if (srcSize - ip < 3) return z1::kDecErrSrcSmall;
            const uint32_t bh = (uint32_t)gb(src + (ip)) | ((uint32_t)gb(src + (ip + 1)) << 8) | ((uint32_t)gb(src + (ip + 2)) << 16);
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
                P.mark(5);
            } else if (btype == z1::kBtRle) {
                if (ip + 1 > srcSize) return z1::kDecErrSrcSmall;
                if (op + bsize > dstCap) return z1::kDecErrDstSmall;
                wave_fill(dst + op, gb(src + (ip)), bsize);
                ip += 1;
                op += bsize;
            } else {
                if (bsize > srcSize - ip) return z1::kDecErrSrcSmall;
                if (bsize > z1::kMaxSrc) return z1::kDecErrCorrupt;
                const uint8_t* blk = src + ip;
                // ---- literals section header
                if (bsize < 1) return z1::kDecErrCorrupt;
                const unsigned ltype = gb(blk + (0)) & 3, sf = (gb(blk + (0)) >> 2) & 3;
                size_t lh, rs, cs = 0;
                bool single = false;
                if (ltype == z1::kSetBasic || ltype == z1::kSetRle) {
                    if (sf == 0 || sf == 2) { lh = 1; rs = gb(blk + (0)) >> 3; }
                    else if (sf == 1) { if (bsize < 2) return z1::kDecErrCorrupt; lh = 2; rs = (gb(blk + (0)) >> 4) + ((size_t)gb(blk + (1)) << 4); }
                    else { if (bsize < 3) return z1::kDecErrCorrupt; lh = 3; rs = (gb(blk + (0)) >> 4) + ((size_t)gb(blk + (1)) << 4) + ((size_t)gb(blk + (2)) << 12); }
                    cs = (ltype == z1::kSetBasic) ? rs : 1;
                } else {
                    if (bsize < 5) return z1::kDecErrCorrupt;
                    const uint32_t lhc = ld32u(blk);
                    if (sf <= 1) { lh = 3; single = (sf == 0); rs = (lhc >> 4) & 0x3FF; cs = (lhc >> 14) & 0x3FF; }
                    else if (sf == 2) { lh = 4; rs = (lhc >> 4) & 0x3FFF; cs = lhc >> 18; }
                    else { lh = 5; rs = (lhc >> 4) & 0x3FFFF; cs = (lhc >> 22) + ((size_t)gb(blk + (4)) << 10); }
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
                P.mark(7);
                if (ltype == z1::kSetBasic) {
                    if (noSeq) wave_copy(litOut, blk + lh, rs);
                    else lit = blk + lh;
                    P.mark(5);
                } else if (ltype == z1::kSetRle) {
                    wave_fill(litOut, gb(blk + (lh)), rs);
                    P.mark(5);
                } else {
                    const uint8_t* hp = blk + lh;
                    size_t remain = cs;
                    if (ltype == z1::kSetCompressed) {
                        unsigned tlNew = 0;
                        const size_t hsz = huf_build_dtable_wave(hp, remain, &tlNew);
                        P.mark(1);
                        if (hsz == 0) return z1::kDecErrCorrupt;
                        hufValid = true;
                        hufTl = tlNew;
                        hp += hsz;
                        remain -= hsz;
                    } else if (!hufValid) {
                        return z1::kDecErrCorrupt;
                    }
                    bool ok = true;
                    if (single) {
                        if (lane == 0) ok = huf_decode1_lane(hufTl, hp, remain, litOut, (uint32_t)rs);
                    } else {
                        ok = huf_decode4_wave(hufTl, hp, remain, litOut, (uint32_t)rs);
                    }
                    if (ballot(!ok)) return z1::kDecErrCorrupt;
                    P.mark(2);
                }
                wave_sync();
                if (noSeq) {
                    op += rs;
                } else {
                    const long r = exec_sequences_wave(seqSrc, seqSize, lit, rs, dst, op, dstCap, frameStart, S, rep, tvalid);
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

}  // namespace pgn
