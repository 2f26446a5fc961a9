// pgn_zenc.h -- one wave compresses one byte stream into a zstd level-1 frame that is byte-identical
// to libzstd 1.4.8/1.4.9 `ZSTD_compress(dst, cap, src, n, 1)` (the call at C5.hpp:337-413).
//
// Data-parallel stages run on all 64 lanes:
//   * the level-1 `fast` match search, speculated 64 visit positions at a time;
//   * literal histograms (LDS atomics, one histogram per Huffman segment);
//   * symbol ranking for the Huffman sort; per-segment bit counts;
//   * Huffman bit packing (prefix sum of code lengths, LDS window, byte flush).
// Serial stages (tree build, weight FSE, sequence FSE) run on lane 0 with the shared zstd1_* code.
#pragma once
#ifndef PGN_AB_SKIP
#define PGN_AB_SKIP 0  // diagnostic builds (tools/ab_skip.sh): 1 no zstd stage, 2 search only, 3 no Huffman, 4 no bit packing, 5 tree only;
                       // PGN_AB_HLOG=h caps the hash log (table-footprint probe)
#endif
#include "pgn_c5.h"
#include "pgn_wave.h"
#include "zstd1_model.h"

namespace pgn {

constexpr int kWinWords = 392;  // 1024 symbols * 12 bits / 32 + carry words
constexpr int kFiltSlots = 512;  // match-search round filter (64 lanes x 2 hashes)

// FSE compression table of the Huffman weight alphabet (<= 13 symbols, tableLog <= 6)
struct WCTable {
    uint32_t tableLog;
    uint16_t stateTable[64];
    uint32_t deltaNbBits[16];
    int32_t deltaFindState[16];
};

// LDS of one encode wave.  The match search and the literal stage never overlap, so their
// workspaces share storage.
struct alignas(16) EncLds {
    union {
        struct {  // match search: hash-slot filter of the current round (bit per lane), the round's visits
            uint64_t filt[kFiltSlots];
            uint32_t vh0[64], vh1[64], vpk[64];
            uint32_t vd0[64], vd1[64];  // the 4 bytes at the round's visits pk and pk + 1
        };
        struct {  // literals; members grouped by lifetime so that each phase's scratch overlays the last
            uint32_t hist2[2][256];  // per-segment histograms, two 16-bit counts per word (histogram -> stream sizes)
            union {
            // the odd lanes' copy of hist2 while the histogram is counted (one word further on, so a
            // byte value counted by both halves of the wave lands in two banks); folded into hist2
            uint32_t hist2x[1 + 2 * 256];
            struct {
            uint8_t nbBits[256];  // tree -> stream sizes
            uint16_t val[256];
            union {
                struct {  // tree build
                    z1::HufNode nodes[2 * 256 + 4];
                    union {
                        uint32_t count[256];  // histogram -> sort (dead before the depths are computed)
                        struct {
                            uint16_t tanc[256];  // tree depths by pointer jumping: ancestor of internal node 256 + i
                            uint16_t tdep[256];  //                                 distance to it
                        };
                    };
                    uint32_t rankLast[16];
                    uint32_t vpr[16];  // valPerRank
                };
                struct {  // table description
                    uint8_t weights[256];
                    uint8_t hdr[256];  // Huffman table description (the FSE form may run to ~210 bytes before it is rejected)
                    WCTable fct;
                    uint8_t fscratch[64];
                    uint32_t wcount[16];  // weight histogram
                    int16_t wnorm[16];
                    uint32_t wcumul[16];
                };
                struct {  // encode (after the table description has left for HBM)
                    uint32_t win[kWinWords];  // output bit window
                    uint32_t cw[256];         // Huffman code | nbBits << 16 (stream sizes -> encode)
                };
            };
            };
            };
        };
        struct {  // sequences section (after the literals section is written)
            z1::FseCTable sct[3];  // ll, of, ml
            uint8_t stsym[512];    // FSE spread scratch
            uint32_t scount[3][64];
            int16_t snorm[64];
            uint32_t scumul[64];
            uint8_t snc[128];      // normalized-count header staging
            uint32_t sv[3][64];    // staged sequences: litLength, mlBase, offset
            uint8_t sc[3][64];     //                   ll, of, ml codes
        };
    };
    uint32_t u[8];
};
__device__ __forceinline__ uint32_t seg_count(const EncLds& L, int k, int s)
{
    return (L.hist2[k >> 1][s] >> (16 * (k & 1))) & 0xFFFFu;
}

// One instance per encode workgroup (the shared codec LDS, pgn_wave.h: every access is a DS instruction).
static_assert(sizeof(EncLds) <= kCodecLdsBytes, "encoder LDS exceeds the codec LDS");
static_assert(__builtin_offsetof(EncLds, hdr) % 4 == 0, "table description words");
#define sEnc (*reinterpret_cast<EncLds*>(sCodecLds))

struct EncScratch {
    uint32_t* ht;        // 2^15 hash-table entries: tag << kTagShift | fingerprint of the 4 bytes | index
    z1::Seq* seqs;       // <= stream/4 + 2 sequences
    uint8_t* codes;      // 3 * (stream/4 + 2)
    uint8_t* lit;        // gathered literals (stream bytes)
    uint8_t* seqSection; // sequences section staging (compress_bound(stream))
    z1::SeqWork* seqWork;
    uint32_t maxSeq;
    uint32_t* huf;       // two Huffman tables (code | nbBits << 16, 256 each): confirmed and candidate
    struct CoopEncCmd __attribute__((address_space(3)))* coop;  // cooperative encode: the post (else null)
};

// ---------------------------------------------------------------------------------------------
// Match search (ZSTD_compressBlock_fast, 1.4.x) speculated over 64 consecutive visits.
// Table entries are (tag << 17) | index; any other tag reads as an empty slot.
// ---------------------------------------------------------------------------------------------
__device__ inline uint32_t wave_match_count(const uint8_t* src, uint32_t a, uint32_t b, uint32_t end)
{
    // 256 bytes per round, four per lane from one unaligned dword load per side (both in flight
    // together: one memory round trip per round; the byte-wise compare with an early exit made four
    // dependent ones).  At the end the lane's dword is taken from end - 4 (or earlier) and shifted, so no
    // byte past `end` is compared; the bytes loaded before a + n lie inside the stream's buffer.
    const uint32_t o = 4u * (uint32_t)lane_id();
    uint32_t n = 0;
    while (a + n < end) {
        const uint32_t len = end - (a + n);
        const uint32_t nv = len > o ? (len - o < 4u ? len - o : 4u) : 0u;  // my bytes inside the stream
        const int32_t so = (int32_t)len - 4 < (int32_t)o ? (int32_t)len - 4 : (int32_t)o;
        const uint32_t wa = ld32u(src + (int64_t)(a + n) + so), wb = ld32u(src + (int64_t)(b + n) + so);
        const uint32_t sh = 8u * (uint32_t)((int32_t)o - so);  // 0, or up to 24 for the end lane
        uint32_t x = nv ? ((wa ^ wb) >> sh) : 0u;
        x &= nv >= 4u ? 0xFFFFFFFFu : ((1u << (8u * nv)) - 1u);
        const uint32_t mism = x ? o + ((uint32_t)__builtin_ctz(x) >> 3) : 0xFFFFFFFFu;
        const uint64_t mm = ballot(mism != 0xFFFFFFFFu);
        if (mm) return n + readlane_u32(mism, __builtin_ctzll(mm));
        if (len <= 256u) return len + n;  // matched to the end
        n += 256;
    }
    return n;
}

// Hash-table entries, 32 bits: a per-slot epoch tag in the top 5 bits (any other tag reads as an
// empty slot; the table is cleared once per kTagEpochs - 1 frames), the index (position + 1) in the
// low idxBits (17 for frames up to 128 KiB, 20 up to 1 MiB, then the frame's bit length up to 26),
// and between them a fingerprint of MEM_read32 at the position (10 bits down to 1).  A candidate whose fingerprint differs
// is no match without reading the stream; one whose fingerprint agrees is confirmed by one read of
// its 4 bytes.  Four bytes per entry keep a slot's table at 2^hashLog x 4 B (32 KiB for the
// hashLog-13 streams), half of an entry that carries the bytes.
constexpr uint32_t kTagShift = 27;
constexpr uint32_t kTagEpochs = 1u << (32 - kTagShift);
// the largest frame source: an index field of 26 bits leaves one fingerprint bit
constexpr uint32_t kMaxIdxBits = 26;
constexpr size_t kMaxFrameBytes = ((size_t)1 << kMaxIdxBits) - 2;
__host__ __device__ inline uint32_t ht_idx_bits(uint32_t frameN)
{
    if (frameN + 2 < (1u << 17)) return 17u;
    if (frameN + 2 < (1u << 20)) return 20u;
    uint32_t b = 21;
    while (b < kMaxIdxBits && frameN + 2 >= (1u << b)) b++;
    return b;
}
// the fingerprint field of the entry for these 4 bytes (bits [idxBits, kTagShift))
__device__ inline uint32_t ht_fp(uint32_t bytes, uint32_t idxBits)
{
    return ((bytes * 0x9E3779B1u) >> (32u - (kTagShift - idxBits))) << idxBits;
}
__device__ inline uint32_t ht_entry(uint32_t tag, uint32_t idx, uint32_t bytes, uint32_t idxBits)
{
    return (tag << kTagShift) | ht_fp(bytes, idxBits) | idx;
}
// A slot's table state between frames (kept in the kernels' epochs array across launches): the
// epoch tag (low 8 bits) and the log2 extent of the entries written since the last clear (above).
// Advances to the epoch of a frame of n bytes; when the tags run out, clears only that extent.
__device__ __forceinline__ void ht_next_epoch(uint32_t* ht, uint32_t& st, uint32_t n)
{
    uint32_t ep = (st & 0xFFu) + 1u, dirty = st >> 8;
    if (ep >= kTagEpochs) {
        for (uint32_t i = (uint32_t)lane_id(); i < ((1u << dirty) >> 2); i += 64) gst<uint4>(ht + 4 * i, make_uint4(0, 0, 0, 0));
        ep = 1;
        dirty = 0;
        wave_sync();
    }
    if (n >= 7) {  // smaller frames are raw blocks and write no entries
        const uint32_t hl = z1::level1_params(n).hashLog;
        dirty = hl > dirty ? hl : dirty;
    }
    st = ep | (dirty << 8);
}

// ZSTD_hashPtr (mls 5 / 6 / 7) over 8 global bytes
__device__ __forceinline__ uint32_t hash_g(const uint8_t* p, unsigned hlog, unsigned mls)
{
    return z1::hash_word(ld64u(p), hlog, mls);
}

// Number of equal bytes going backwards from a-1 / b-1, at most `lim` (wave-parallel, 64 per step)
__device__ inline uint32_t wave_back_count(const uint8_t* src, uint32_t a, uint32_t b, uint32_t lim)
{
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t n = 0;
    while (n < lim) {
        const uint32_t o = n + lane + 1;
        const bool diff = (o <= lim) && gb(src + a - o) != gb(src + b - o);
        const uint64_t m = ballot(diff || o > lim);
        if (m) return n + (uint32_t)__builtin_ctzll(m);
        n += 64;
    }
    return lim;
}

// The no-match visit recurrence of ZSTD_compressBlock_fast (ip += ((ip - anchor) >> 7) + 2), as
// e = ip - anchor + 256 -> e + (e >> 7), only ever starts at e = 256 (a round after a match or a
// repcode run: ip == anchor) or 257 (the first block of a frame: ip = 1, anchor = 0).  Both chains
// are tabulated once (constant memory, read through the caches), so a round's 64 visit positions are
// one coalesced load instead of 64 dependent scalar steps.
constexpr int kChainLen = 1344;
struct VisitChains {
    uint32_t e[2][kChainLen];
};
constexpr VisitChains make_visit_chains()
{
    VisitChains c{};
    for (int s = 0; s < 2; s++) {
        uint32_t e = 256u + (uint32_t)s;
        for (int i = 0; i < kChainLen; i++) {
            c.e[s][i] = e;
            e += e >> 7;
        }
    }
    return c;
}
constexpr VisitChains kVisitChainsHost = make_visit_chains();
// a round reads entries ci .. ci + 64; the chains must outrun any block (e <= 2^20 + 256)
static_assert(kVisitChainsHost.e[0][kChainLen - 65] > (1u << 20) + 512u, "visit chain too short");
__constant__ VisitChains kVisitChains = make_visit_chains();

// No-match certificate (single-block frames).  Until its first match ZSTD_compressBlock_fast visits
// a data-independent chain of positions (two per iteration, ip0 and ip0 + 1), tests the repcode at
// ip0 + 2 and, for each visited position, the table's entry for its hash: the latest visited position
// with that hash.  So if no iteration's repcode holds and no two visited positions share their hash
// and their first 4 bytes, the search finds nothing: the block is all literals (nbSeq 0, repeat
// offsets unchanged), whatever the table holds -- and the table (a frame starts with an empty one,
// tagged per frame) need not be read or written at all.  The pairs are found with a blocked Bloom
// filter over the keys (hash, 4 bytes) in the codec LDS (the search's own LDS is not yet live): a key
// sets six bits of one 64-bit word with one LDS atomic OR, and finds its bits already set when an
// equal key came before it (the atomics on one word are ordered, also between the lanes of one
// instruction); any repcode hit or key whose bits were all set -- an equal key or a false positive,
// about 4 % of 100,000-sample M streams -- returns false and the exact search runs.  For noise streams
// (the C5 S / M / Llow streams) this replaces the search's table round trips, the bulk of the
// encoder's HBM bytes.
constexpr uint32_t kCertWords = kCodecLdsBytes / 8;  // 64-bit filter words
constexpr uint32_t kCertKeys = 2048;                 // at most this many keys (false positives stay rare)
__device__ __forceinline__ uint32_t fmix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
typedef __attribute__((address_space(3))) uint64_t lds_u64;
// one key into the filter; true if its six bits were all set before
__device__ __forceinline__ bool cert_insert(lds_u64* words, uint32_t x)
{
    const uint32_t a = fmix32(x), b = fmix32(x ^ 0x5BD1E995u);
    const uint64_t m = (1ull << (a & 63u)) | (1ull << ((a >> 6) & 63u)) | (1ull << ((a >> 12) & 63u)) |
                       (1ull << ((a >> 18) & 63u)) | (1ull << ((a >> 24) & 63u)) | (1ull << (b & 63u));
    const uint32_t w = (b >> 6) & (kCertWords - 1u);
    const uint64_t old = __hip_atomic_fetch_or(words + w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (old & m) == m;
}
static_assert((kCertWords & (kCertWords - 1)) == 0, "filter words: a power of two");
__device__ __noinline__ bool no_match_certificate(const uint8_t* __restrict__ src, uint32_t n, unsigned hlog, unsigned mls,
                                                  uint32_t off1)
{
    const uint32_t lane = (uint32_t)lane_id();
    src = uni(src);
    n = uni(n);
    hlog = uni(hlog);
    mls = uni(mls);
    off1 = uni(off1);
    lds_u64* words = (lds_u64*)sCodecLds;
    for (uint32_t i = lane; i < kCertWords; i += 64) words[i] = 0;
    lds_sync();
    const int32_t ilimit = (int32_t)n - 8;
    const uint32_t* E = kVisitChains.e[1];  // the first block of a frame: ip0 = 1, anchor = 0
    // software pipeline: a round's bytes were loaded during the round before, and its positions
    // two rounds ahead (the chain is data-independent), so a round waits on no memory round trip
    auto loads = [&](int32_t p, uint64_t& v, uint32_t& r) {
        if (p + 1 < ilimit) {
            v = ld64u(src + p);
            r = off1 > 0 ? ld32u(src + p + 2 - (int32_t)off1) : 0u;
        }
    };
    int32_t pk = (int32_t)E[lane] - 256, pkN = (int32_t)E[64 + lane] - 256;
    uint64_t v8 = 0;
    uint32_t rw = 0;
    loads(pk, v8, rw);
    for (uint32_t ci = 0;; ci += 64) {
        if (2 * (ci + 64) > kCertKeys) return false;  // too many keys: the exact search decides
        uint64_t v8N = 0;
        uint32_t rwN = 0;
        loads(pkN, v8N, rwN);
        const int32_t pkNN = (int32_t)E[ci + 128 + lane] - 256;
        const bool valid = pk + 1 < ilimit;
        bool bad = false;
        if (valid) {
            bad = off1 > 0 && rw == (uint32_t)(v8 >> 16);
            const uint32_t h0 = z1::hash_word(v8, hlog, mls), h1 = z1::hash_word(v8 >> 8, hlog, mls);
            // ip0's key before ip1's: a lane's two keys are ordered too
            if (cert_insert(words, (uint32_t)v8 ^ (h0 * 0x9E3779B1u))) bad = true;
            if (cert_insert(words, (uint32_t)(v8 >> 8) ^ (h1 * 0x9E3779B1u))) bad = true;
        }
        if (ballot(bad)) return false;
        if (ballot(!valid)) return true;  // the chain has left the block
        pk = pkN;
        pkN = pkNN;
        v8 = v8N;
        rw = rwN;
    }
}

// Match search (ZSTD_compressBlock_fast, libzstd 1.4.x) speculated over 64 consecutive visits.
// The visit positions follow a data-independent recurrence until a match is found, so lane k takes
// visit k of the round: it hashes its two positions, reads the table (entries (tag << 17) | idx,
// another tag reads as empty) unless an earlier visit of the round wrote the same slot, and tests
// the repcode and both candidates; a ballot finds the first hit.  Visits before it commit their
// table writes (the last writer of a slot wins), the hit is processed as the serial loop does, and
// the next round starts after it.  Same-slot writers inside a round are found through an LDS filter
// (one bit per lane per slot), checked exactly only for the lanes whose filter slots collide.
// Searches the block [start, end) of src (table and positions frame-wide, zstd1_model.h
// fast_search_serial); rep0 / rep1 are the confirmed repeat offsets on entry.
struct SearchOut {
    uint32_t nbSeq, lastLL, rep0, rep1, rounds;
    uint32_t candIters;  // profile builds: wave iterations of the same-slot loops
};
__device__ __noinline__ SearchOut fast_search_wave(const uint8_t* __restrict__ src, uint32_t start, uint32_t end, unsigned hlog,
                                                   unsigned mls, uint32_t* __restrict__ ht, uint32_t tag,
                                                   z1::Seq* __restrict__ seqs, uint32_t rep0, uint32_t rep1, uint32_t idxBits,
                                                   uint32_t lowIdx, uint32_t maxRep, bool single)
{
    EncLds& L = sEnc;
    const uint32_t lane = (uint32_t)lane_id();
    src = uni(src);
    start = uni(start);
    end = uni(end);
    hlog = uni(hlog);
#ifdef PGN_AB_HLOG
    hlog = hlog > PGN_AB_HLOG ? PGN_AB_HLOG : hlog;  // diagnostic: smaller tables (other matches, not parity)
#endif
    mls = uni(mls);
    ht = uni(ht);
    tag = uni(tag);
    seqs = uni(seqs);
    rep0 = uni(rep0);
    rep1 = uni(rep1);
    idxBits = uni(idxBits);
    const uint32_t idxMask = (1u << idxBits) - 1u, fpMask = ((1u << kTagShift) - 1u) & ~idxMask;
    const int32_t iend = (int32_t)end, ilimit = (int32_t)end - 8;
    int32_t ip0 = (int32_t)start + (start == 0 ? 1 : 0), anchor = (int32_t)start;
    // ZSTD_compressBlock_fast_generic: repeat offsets beyond the window at the first position are
    // invalidated (maxRep); table candidates must lie above the block's lowest prefix index lowIdx
    // (1 for a frame within its window; ZSTD_getLowestPrefixIndex of the block's end above it)
    lowIdx = uni(lowIdx);
    maxRep = uni(maxRep);
    single = __builtin_amdgcn_readfirstlane((int)single) != 0;
    uint32_t off1 = rep0, off2 = rep1, offSaved = 0;
    if (off2 > maxRep) { offSaved = off2; off2 = 0; }
    if (off1 > maxRep) { offSaved = off1; off1 = 0; }
#ifdef PGN_NO_CERT  // A/B builds: the exact search only
    single = false;
#endif
    if (single && no_match_certificate(src, end, hlog, mls, off1)) {  // the whole frame is one literals block
        SearchOut r;
        r.nbSeq = 0;
        r.lastLL = end - start;
        r.rep0 = off1 ? off1 : offSaved;
        r.rep1 = off2 ? off2 : offSaved;
        r.rounds = 0;
        r.candIters = 0;
        return r;
    }
    uint32_t nbSeq = 0, rounds = 0, candIters = 0;
    const uint64_t below = (1ull << lane) - 1ull, above = ~below & ~(1ull << lane);
    for (int i = (int)lane; i < kFiltSlots; i += 64) L.filt[i] = 0;  // shares storage with the literal stage
    lds_sync();
    // positions of the 64 visits at chain index ci (the no-match recurrence, tabulated in
    // kVisitChains; the chain restarts at index 0 after every match)
    uint32_t chain = (start == 0) ? 1u : 0u, ci = 0;
    auto positions = [&](uint32_t c, int32_t& pkOut, int32_t& pNextOut) {
        const uint32_t* E = kVisitChains.e[chain];
        pkOut = (int32_t)E[c + lane] + (anchor - 256);
        pNextOut = (int32_t)E[c + 64] + (anchor - 256);
    };
    int32_t pk = 0, pNext = 0;
    uint64_t v8 = 0;    // bytes pk .. pk+7: both hashes and the current-position words
    uint32_t repw = 0;  // bytes at pk + 2 - off1 (repcode candidate)
    auto loads = [&](int32_t p, uint64_t& v, uint32_t& r) {
        if (p + 1 < ilimit) {
            v = ld64u(src + p);
            r = (off1 > 0) ? ld32u(src + p + 2 - (int32_t)off1) : 0u;
        }
    };
    bool havePk = false;  // pk / pNext / v8 / repw already hold this round's visits (from the last round)
    while (ip0 + 1 < ilimit) {
        rounds++;
        if (!havePk) {
            positions(ci, pk, pNext);
            loads(pk, v8, repw);
        }
        havePk = false;
        const bool valid = (pk + 1 < ilimit);
        uint32_t h0 = 0xFFFFFFFFu, h1 = 0xFFFFFFFEu;
        uint32_t t0 = 0, t1 = 0;
        uint64_t M0 = 0, M1 = 0;
        if (valid) {
            h0 = z1::hash_word(v8, hlog, mls);
            h1 = z1::hash_word(v8 >> 8, hlog, mls);
            t0 = gld<uint32_t>(ht + h0);
            t1 = gld<uint32_t>(ht + h1);
            atomicOr((unsigned long long*)&L.filt[h0 & (kFiltSlots - 1)], (unsigned long long)(1ull << lane));
            atomicOr((unsigned long long*)&L.filt[h1 & (kFiltSlots - 1)], (unsigned long long)(1ull << lane));
        }
        L.vh0[lane] = h0;
        L.vh1[lane] = h1;
        L.vpk[lane] = (uint32_t)pk;
        L.vd0[lane] = (uint32_t)v8;
        L.vd1[lane] = (uint32_t)(v8 >> 8);
        // the next round's visits and their bytes, assuming this one finds no match (overlaps the
        // table reads)
        int32_t pkN, pNextN;
        positions(ci + 64, pkN, pNextN);
        uint64_t v8N = 0;
        uint32_t repwN = 0;
        loads(pkN, v8N, repwN);
        lds_sync();
        if (valid) {
            M0 = L.filt[h0 & (kFiltSlots - 1)];
            M1 = L.filt[h1 & (kFiltSlots - 1)];
        }
        lds_sync();
        if (valid) {
            L.filt[h0 & (kFiltSlots - 1)] = 0;
            L.filt[h1 & (kFiltSlots - 1)] = 0;
        }
        // value each slot holds at my visit: the latest earlier writer in this round (its bytes known
        // exactly), else the table (its fingerprint)
        const uint32_t fp0 = ht_fp((uint32_t)v8, idxBits), fp1 = ht_fp((uint32_t)(v8 >> 8), idxBits);
        uint32_t m0 = ((t0 >> kTagShift) == tag) ? (t0 & idxMask) : 0u;
        uint32_t m1 = ((t1 >> kTagShift) == tag) ? (t1 & idxMask) : 0u;
        bool fpok0 = ((t0 ^ fp0) & fpMask) == 0, fpok1 = ((t1 ^ fp1) & fpMask) == 0;
        bool fw0 = false, fw1 = false;
        uint32_t d0 = 0, d1 = 0;
#ifdef PGN_PROFILE
        uint32_t myIt = 0;
#endif
        for (uint64_t cand = M0 & below; cand;) {
#ifdef PGN_PROFILE
            myIt++;
#endif
            const int jj = 63 - __builtin_clzll(cand);
            const uint32_t pj = L.vpk[jj];
            if (L.vh1[jj] == h0) { m0 = pj + 2; d0 = L.vd1[jj]; fw0 = true; break; }
            if (L.vh0[jj] == h0) { m0 = pj + 1; d0 = L.vd0[jj]; fw0 = true; break; }
            cand &= ~(1ull << jj);
        }
        for (uint64_t cand = M1 & below; cand;) {
#ifdef PGN_PROFILE
            myIt++;
#endif
            const int jj = 63 - __builtin_clzll(cand);
            const uint32_t pj = L.vpk[jj];
            if (L.vh1[jj] == h1) { m1 = pj + 2; d1 = L.vd1[jj]; fw1 = true; break; }
            if (L.vh0[jj] == h1) { m1 = pj + 1; d1 = L.vd0[jj]; fw1 = true; break; }
            cand &= ~(1ull << jj);
        }
        bool rep = false, c0 = false, c1 = false;
        if (valid) {
            rep = (off1 > 0) && (repw == (uint32_t)(v8 >> 16));
            c0 = (m0 > lowIdx) && (fw0 ? d0 == (uint32_t)v8 : fpok0);
            c1 = (m1 > lowIdx) && (fw1 ? d1 == (uint32_t)(v8 >> 8) : fpok1);
        }
#ifdef PGN_PROFILE
        candIters += wave_max(myIt);
#endif
        // The first hit decides the round.  A table candidate there has only its fingerprint checked,
        // so its bytes are compared by counting the match forward from its first byte -- the count
        // the match needs anyway, so a true match costs no extra read; a false candidate is dropped
        // and the next hit taken.
        uint64_t hits = ballot(rep || c0 || c1);
        uint32_t fwdKnown = 0;  // forward length of the chosen table candidate from its first byte
        {
            const uint64_t fwb0 = ballot(fw0), fwb1 = ballot(fw1);
            while (hits) {
                const int ff = __builtin_ctzll(hits);
                if ((ballot(rep) >> ff) & 1) break;
                const bool isC0 = (ballot(c0) >> ff) & 1;
                if (((isC0 ? fwb0 : fwb1) >> ff) & 1) break;  // an earlier visit's write: bytes compared exactly
                const uint32_t mf = readlane_u32(isC0 ? m0 : m1, ff);
                const uint32_t ipc = readlane_u32((uint32_t)pk, ff) + (isC0 ? 0u : 1u);
                const uint32_t nm = wave_match_count(src, ipc, mf - 1, (uint32_t)iend);
                if (nm >= 4) {
                    fwdKnown = nm;
                    break;
                }
                if ((int)lane == ff) {
                    if (isC0) c0 = false;
                    else c1 = false;
                }
                hits = ballot(rep || c0 || c1);
            }
        }
        const uint64_t vmask = ballot(valid);
        const int f = hits ? __builtin_ctzll(hits) : 64;
        const int lastCommit = hits ? f : (63 - __builtin_clzll(vmask));
        if (valid && (int)lane <= lastCommit) {
            // my write survives unless a later committed visit of the round writes the same slot
            const uint64_t upto = (lastCommit >= 63) ? ~0ull : ((1ull << (lastCommit + 1)) - 1ull);
            bool w0 = (h0 != h1), w1 = true;
            for (uint64_t cand = M0 & above & upto; cand && w0;) {
                const int jj = __builtin_ctzll(cand);
                if (L.vh0[jj] == h0 || L.vh1[jj] == h0) w0 = false;
                cand &= cand - 1;
            }
            for (uint64_t cand = M1 & above & upto; cand && w1;) {
                const int jj = __builtin_ctzll(cand);
                if (L.vh0[jj] == h1 || L.vh1[jj] == h1) w1 = false;
                cand &= cand - 1;
            }
            if (w0) gst<uint32_t>(ht + h0, (tag << kTagShift) | fp0 | ((uint32_t)pk + 1));
            if (w1) gst<uint32_t>(ht + h1, (tag << kTagShift) | fp1 | ((uint32_t)pk + 2));
        }
        lds_sync();
        if (!hits) {
            wave_sync();
            if (vmask == ~0ull) {
                ip0 = pNext;
                ci += 64;
                pk = pkN;
                pNext = pNextN;
                v8 = v8N;
                repw = repwN;
                havePk = true;
                continue;
            }
            break;
        }
        // the match found at visit f, processed exactly as the serial loop does
        const int32_t ipf = (int32_t)L.vpk[f];
        const bool repf = (ballot(rep) >> f) & 1, c0f = (ballot(c0) >> f) & 1;
        const uint32_t m0f = readlane_u32(m0, f), m1f = readlane_u32(m1, f);
        const uint32_t cur0 = (uint32_t)ipf + 1;
        int32_t ipm, match0;
        uint32_t mLength, offcode;
        if (repf) {
            const int32_t ip2 = ipf + 2;
            mLength = (gb(src + (ip2 - 1)) == gb(src + (ip2 - (int32_t)off1 - 1))) ? 1u : 0u;
            ipm = ip2 - (int32_t)mLength;
            match0 = ipm - (int32_t)off1;
            mLength += 4;
            offcode = 0;
        } else {
            if (c0f) { ipm = ipf; match0 = (int32_t)m0f - 1; }
            else { ipm = ipf + 1; match0 = (int32_t)m1f - 1; }
            off2 = off1;
            off1 = (uint32_t)(ipm - match0);
            offcode = off1 + 2;
            mLength = 4;
            const int32_t room = match0 - ((int32_t)lowIdx - 1);  // down to the window's first position
            const int32_t lim = (ipm - anchor) < room ? (ipm - anchor) : room;
            const uint32_t back = lim > 0 ? wave_back_count(src, (uint32_t)ipm, (uint32_t)match0, (uint32_t)lim) : 0u;
            ipm -= (int32_t)back;
            match0 -= (int32_t)back;
            mLength += back;
        }
        // (the forward part starts 4 bytes past the candidate, whatever the backward extension)
        mLength += fwdKnown ? fwdKnown - 4u
                            : wave_match_count(src, (uint32_t)ipm + mLength, (uint32_t)match0 + mLength, (uint32_t)iend);
        if (lane == 0) {
            seqs[nbSeq].litLength = (uint32_t)(ipm - anchor);
            seqs[nbSeq].offset = offcode + 1;
            seqs[nbSeq].mlBase = mLength - 3;
        }
        nbSeq++;
        ip0 = ipm + (int32_t)mLength;
        anchor = ip0;
        chain = 0;
        ci = 0;
        if (ip0 <= ilimit) {
            // what this tail and the next round read, in flight together: the two new table entries'
            // words, the repeat-offset check's words and the next round's visits (valid unless a
            // repeat match moves the anchor and swaps the offsets) -- one memory round trip, not three
            uint64_t wa = 0, wb = 0;
            if (lane == 0) {
                wa = ld64u(src + cur0 + 1);
                wb = ld64u(src + ip0 - 2);
            }
            uint32_t rc0 = 0, rc1 = 0;
            if (off2 > 0) {
                rc0 = ld32u(src + ip0);
                rc1 = ld32u(src + ip0 - (int32_t)off2);
            }
            positions(0, pk, pNext);
            loads(pk, v8, repw);
            havePk = true;
            if (lane == 0) {
                gst<uint32_t>(ht + z1::hash_word(wa, hlog, mls), ht_entry(tag, cur0 + 2, (uint32_t)wa, idxBits));
                gst<uint32_t>(ht + z1::hash_word(wb, hlog, mls), ht_entry(tag, (uint32_t)(ip0 - 2) + 1, (uint32_t)wb, idxBits));
            }
            if (off2 > 0) {
                bool firstRep = true;
                while ((ip0 <= ilimit) &&
                       (firstRep ? rc0 == rc1 : ld32u(src + ip0) == ld32u(src + ip0 - (int32_t)off2))) {
                    firstRep = false;
                    havePk = false;  // the anchor moves and the offsets swap
                    const uint32_t rLength = wave_match_count(src, (uint32_t)ip0 + 4, (uint32_t)ip0 + 4 - off2, (uint32_t)iend) + 4;
                    const uint32_t t = off2;
                    off2 = off1;
                    off1 = t;
                    if (lane == 0) {
                        const uint64_t wr = ld64u(src + ip0);
                        gst<uint32_t>(ht + z1::hash_word(wr, hlog, mls), ht_entry(tag, (uint32_t)ip0 + 1, (uint32_t)wr, idxBits));
                        seqs[nbSeq].litLength = 0;
                        seqs[nbSeq].offset = 1;
                        seqs[nbSeq].mlBase = rLength - 3;
                    }
                    nbSeq++;
                    ip0 += (int32_t)rLength;
                    anchor = ip0;
                }
            }
        }
        wave_sync();
    }
    SearchOut r;
    r.nbSeq = nbSeq;
    r.lastLL = (uint32_t)(iend - anchor);
    r.rep0 = off1 ? off1 : offSaved;
    r.rep1 = off2 ? off2 : offSaved;
    r.rounds = rounds;
    r.candIters = candIters;
    return r;
}

// ---------------------------------------------------------------------------------------------
// Huffman bit packing of one segment: symbols are written last-to-first (HUF_compress1X order), so
// emission r takes symbol src[len-1-r] and its bit position is the sum of the code lengths emitted
// before it.  A step emits 1024 symbols, 16 per lane from one 16-byte load; lane code groups are
// OR-ed into an LDS bit window at their prefix-sum offsets, and the window's complete words leave
// as coalesced dword stores.
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ void huf_encode_segment_wave(uint8_t* __restrict__ out, const uint8_t* __restrict__ src, uint32_t len,
                                                     uint32_t totalBits, lds_u32* win)
{
    const uint32_t lane = (uint32_t)lane_id();
    out = uni(out);
    src = uni(src);
    len = uni(len);
    totalBits = uni(totalBits);
    const uint32_t* cw = sEnc.cw;
    for (uint32_t w = lane; w < (uint32_t)kWinWords; w += 64) win[w] = 0;
    lds_sync();
    uint32_t winLo = 0;   // bit offset of win[0] (multiple of 32)
    uint32_t bitBase = 0; // bits emitted before this step
    // the next step's 16-byte block is loaded one step ahead
    uint4 nv = make_uint4(0, 0, 0, 0);
    if ((int32_t)len - 16 - (int32_t)(16 * lane) >= 0) nv = gld<uint4>(src + (len - 16 - 16 * lane));
    // a step of 1024 emissions; FULL (every lane's 16 emissions exist: all but the last step) reads
    // the code table without per-symbol masks (predicated LDS reads cost an exec-mask round per symbol)
    auto step = [&](auto FULL, uint32_t r0) {
        // my 16 emissions r0 + 16*lane + j are bytes len-1-r of src: one 16-byte block, reversed
        const int32_t a = (int32_t)len - 16 - (int32_t)(r0 + 16 * lane);
        uint32_t wv[4];
        if (FULL || a >= 0) {
            const uint4 v = nv;
            wv[0] = v.x; wv[1] = v.y; wv[2] = v.z; wv[3] = v.w;
            if (a - 1024 >= 0) nv = gld<uint4>(src + (a - 1024));
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t x = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int32_t i = a + 4 * q + b;
                    if (i >= 0) x |= (uint32_t)gb(src + i) << (8 * b);
                }
                wv[q] = x;
            }
        }
        const int32_t nvalid = (int32_t)len - (int32_t)(r0 + 16 * lane);  // emissions of mine (may be <= 0 or > 16)
        uint64_t grp[4];
        uint32_t gnb[4];
        uint32_t myBits = 0;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint64_t acc = 0;
            uint32_t n = 0;
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int j = 4 * g + jj;
                const uint32_t sym = (wv[(15 - j) >> 2] >> (8 * ((15 - j) & 3))) & 0xFFu;
                uint32_t cwj = cw[sym];
                if (!FULL) cwj = (j < nvalid) ? cwj : 0u;
                acc |= (uint64_t)(cwj & 0xFFFFu) << n;
                n += cwj >> 16;
            }
            grp[g] = acc;
            gnb[g] = n;
            myBits += n;
        }
        const uint32_t incl = wave_incl_sum(myBits);
        const uint32_t stepBits = readlane_u32(incl, 63);
        uint32_t pos = bitBase + (incl - myBits) - winLo;  // window-relative bit position
        // a group (<= 44 bits) at bit pos touches words w .. w + 2: three unconditional ORs (of zero
        // where it does not reach), no branches
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t w = pos >> 5, sh = pos & 31;
            const uint64_t lo = grp[g] << sh;
            __hip_atomic_fetch_or(&win[w], (uint32_t)lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_or(&win[w + 1], (uint32_t)(lo >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_or(&win[w + 2], (uint32_t)((grp[g] >> 32) >> (32 - sh)), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
            pos += gnb[g];
        }
        lds_sync();
        const uint32_t endRel = bitBase + stepBits - winLo;
        const uint32_t complete = endRel >> 5;
        uint8_t* o = out + (winLo >> 3);
        // complete words leave and are cleared in one pass; the partial word moves to the front
        const uint32_t carry = win[complete];
        for (uint32_t w = lane; w <= complete; w += 64) {
            const uint32_t v = win[w];
            // the packed bits go to the blob once: non-temporal (encode -0.6 % in A/B, r05ent)
            if (w < complete) __builtin_nontemporal_store(v, (__attribute__((address_space(1))) uint32_t*)(o + 4 * w));
            win[w] = 0u;
        }
        if (lane == 0) win[0] = carry;
        lds_sync();
        winLo += complete * 32;
        bitBase += stepBits;
    };
    uint32_t r0 = 0;
    for (; r0 + 1024 <= len; r0 += 1024) step(std::true_type{}, r0);
    if (r0 < len) step(std::false_type{}, r0);
    // end mark, then the last partial bytes
    if (lane == 0) {
        const uint32_t rel = totalBits - winLo;
        win[rel >> 5] |= 1u << (rel & 31);
    }
    lds_sync();
    const uint32_t nbytes = ((totalBits + 8) >> 3) - (winLo >> 3);
    uint8_t* o = out + (winLo >> 3);
    for (uint32_t b = lane; b < nbytes; b += 64) gst<uint8_t>(o + b, (uint8_t)(win[b >> 2] >> (8 * (b & 3))));
    lds_sync();
}

// ---------------------------------------------------------------------------------------------
// Cooperative encode (small batches, enc_zstd_coop_kernel): a workgroup of kCoopEncWaves waves per
// stream.  Wave 0 runs zstd1_compress_wave<true>; a four-segment literals section's histograms and
// its bit packing are posted here, and wave k does segment k (its own bit window); the rest is wave 0's.
// ---------------------------------------------------------------------------------------------
constexpr int kCoopEncWaves = 4;
struct CoopEncCmd {
    uint32_t op;  // 0: done, 1: segment histograms, 2: segment bit packing
    uint32_t n, segSize;
    const uint8_t* lit;
    uint8_t* out[4];
    uint32_t bits[4];
};
typedef __attribute__((address_space(3))) CoopEncCmd lds_enc_cmd;

// the histogram of literals segment k ([k segSize, min((k + 1) segSize, n))) into sEnc.hist2, whose
// other segments other waves add at the same time (LDS atomics)
__device__ __noinline__ void hist_segment_wave(const uint8_t* __restrict__ lit, uint32_t n, uint32_t segSize, uint32_t k)
{
    EncLds& L = sEnc;
    const uint32_t lane = (uint32_t)lane_id();
    lit = uni(lit);
    n = uni(n);
    segSize = uni(segSize);
    k = uni(k);
    const uint32_t a0 = k * segSize, a1 = (k + 1) * segSize < n ? (k + 1) * segSize : n;
    uint32_t* h = &L.hist2[k >> 1][0];
    const uint32_t inc = 1u << (16 * (k & 1));
    for (uint32_t i0 = a0 + 16u * lane; i0 < a1; i0 += 4096) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 1024u * (uint32_t)u;
            if (i + 16 <= a1) {
                v[u] = gld<uint4>(lit + i);
            } else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (uint32_t b = 0; b < 16; b++)
                    if (i + b < a1) w[b >> 2] |= (uint32_t)gb(lit + i + b) << (8 * (b & 3));
                v[u] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 1024u * (uint32_t)u;
            const uint32_t wd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            if (i + 16 <= a1) {
#pragma unroll
                for (int b = 0; b < 16; b++) atomicAdd(h + ((wd[b >> 2] >> (8 * (b & 3))) & 0xFFu), inc);
            } else {
                for (uint32_t b = 0; b < 16; b++)
                    if (i + b < a1) atomicAdd(h + ((wd[b >> 2] >> (8 * (b & 3))) & 0xFFu), inc);
            }
        }
    }
}

// waves 1..3 of a cooperative encode workgroup
__device__ __noinline__ void coop_enc_helper_wave(uint32_t wid, lds_enc_cmd* cmd, lds_u32* win)
{
    while (true) {
        __syncthreads();  // B1: a job (or done) is posted
        const uint32_t op = cmd->op;
        if (op == 0) break;
        if (op == 1) hist_segment_wave(cmd->lit, cmd->n, cmd->segSize, wid);
        else {
            const uint32_t a = cmd->segSize * wid, e = wid == 3 ? cmd->n : a + cmd->segSize;
            huf_encode_segment_wave(cmd->out[wid], cmd->lit + a, e - a, cmd->bits[wid], win);
        }
        __syncthreads();  // B2
    }
}
__device__ __forceinline__ void coop_enc_finish(lds_enc_cmd* cmd)
{
    if (lane_id() == 0) cmd->op = 0;
    __syncthreads();  // B1 with op 0
}

// ---------------------------------------------------------------------------------------------
// Huffman tree on the wave: HUF_buildCTable_wksp + HUF_setMaxHeight (libzstd 1.4.x) over the sorted
// leaves L.nodes[1 + r] (count desc, symbol asc; zero past the last symbol).  The two-queue merge
// runs wave-uniform (scalar control, look-ahead registers for both queue heads); depths come from
// pointer jumping over the parent links; the rank boundaries of HUF_setMaxHeight and the canonical
// codes from ballots.  Writes L.nbBits / L.val per symbol; returns the largest code length.
// nnz = number of symbols with a nonzero count (>= 2).
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ uint32_t huf_tree_wave(uint32_t maxSym, uint32_t maxNbBits, uint32_t nnz, PhaseProf& P)
{
    EncLds& L = sEnc;
    const int lane = lane_id();
    maxSym = uni(maxSym);
    maxNbBits = uni(maxNbBits);
    nnz = uni(nnz);
    z1::HufNode* hn = L.nodes + 1;
    constexpr int kStart = z1::kHufStartNode;
    const int nonNullRank = (int)nnz - 1;
    const int nodeRoot = kStart + nonNullRank - 1;
    P.count(2);
    L.nodes[0].count = 1u << 31;  // huffNode0[0]: barrier below the leaves
    // ---- create parents in rounds of independent merges.  The two-queue merge (leaves ascending
    // from lowS down, nodes hn[lowN .. nodeNb) in creation order, a leaf taken only when strictly
    // smaller) creates nodes of nondecreasing count, so with s = the sum of the next two picks, every
    // queued node (<= s) and every leaf < s is picked before the node of count s is: those t
    // elements, merged in pick order, form floor(t / 2) nodes at once -- node nodeNb + k from picks
    // 2k and 2k + 1, exactly the serial loop's nodes.  An odd last element starts the next round.
    // Pick positions: a leaf's is its rank plus the queued nodes <= it, a node's its rank plus the
    // leaves < it (binary searches over the two sorted runs in LDS).
    uint32_t* pickVal = L.count;  // dead after the sort
    int lowS = nonNullRank, lowN = kStart, nodeNb = kStart;
    uint32_t rounds = 0;
    while (nodeNb <= nodeRoot) {
        rounds++;
        uint32_t s;
        {
            const uint32_t S0 = lowS >= 0 ? hn[lowS].count : (1u << 31);
            const uint32_t S1 = lowS >= 1 ? hn[lowS - 1].count : (1u << 31);
            const uint32_t Q0 = lowN < nodeNb ? hn[lowN].count : (1u << 30);
            const uint32_t Q1 = lowN + 1 < nodeNb ? hn[lowN + 1].count : (1u << 30);
            s = (S0 < Q0) ? S0 + (S1 < Q0 ? S1 : Q0) : Q0 + (S0 < Q1 ? S0 : Q1);
        }
        const uint32_t nq = (uint32_t)(nodeNb - lowN);
        // leaves < s: a run ending at lowS (ascending rank i = leaf lowS - i)
        const int leafSlots = (lowS + 64) >> 6;
        uint32_t nl = 0;
        uint32_t lv[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            lv[j] = 0xFFFFFFFFu;
            if (j < leafSlots) {
                const int i = lane + 64 * j;
                if (i <= lowS) lv[j] = hn[lowS - i].count;
                nl += (uint32_t)__builtin_popcountll(ballot(lv[j] < s));
            }
        }
        nl = uni(nl);
        const uint32_t t = nl + nq, pairs = t >> 1, used = 2 * pairs;
        uint32_t usedLeaves = 0;
        const uint32_t stN = nq ? (1u << (31 - __builtin_clz(nq))) : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (j < leafSlots) {
                const uint32_t i = (uint32_t)lane + 64u * (uint32_t)j;
                uint32_t lo = 0;
                // branch-free: a probe past the run is clamped to its last element (the predicate is
                // monotone, so taking the clamped position when it holds is still exact)
                for (uint32_t st = stN; st; st >>= 1) {
                    const uint32_t k = lo + st, kc = k < nq ? k : nq;
                    lo = hn[lowN + (int)kc - 1].count <= lv[j] ? kc : lo;
                }
                const uint32_t pos = i + lo;
                const bool take = i < nl && pos < used;
                if (take) {
                    hn[lowS - (int)i].parent = (uint16_t)(nodeNb + (int)(pos >> 1));
                    pickVal[pos] = lv[j];
                }
                usedLeaves += (uint32_t)__builtin_popcountll(ballot(take));
            }
        }
        const uint32_t stL = nl ? (1u << (31 - __builtin_clz(nl))) : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (64u * (uint32_t)j < nq) {
                const uint32_t m = (uint32_t)lane + 64u * (uint32_t)j;
                if (m < nq) {
                    const uint32_t v = hn[lowN + (int)m].count;
                    uint32_t lo = 0;
                    for (uint32_t st = stL; st; st >>= 1) {
                        const uint32_t k = lo + st, kc = k < nl ? k : nl;
                        lo = hn[lowS - (int)kc + 1].count < v ? kc : lo;
                    }
                    const uint32_t pos = m + lo;
                    if (pos < used) {
                        hn[lowN + (int)m].parent = (uint16_t)(nodeNb + (int)(pos >> 1));
                        pickVal[pos] = v;
                    }
                }
            }
        }
        lds_sync();
        for (uint32_t k = (uint32_t)lane; k < pairs; k += 64) hn[nodeNb + (int)k].count = pickVal[2 * k] + pickVal[2 * k + 1];
        lds_sync();
        usedLeaves = uni(usedLeaves);
        lowS -= (int)usedLeaves;
        lowN += (int)(used - usedLeaves);
        nodeNb += (int)pairs;
    }
    P.count(3, rounds);
    lds_sync();
    P.mark(11);
    // ---- depths of the internal nodes: pointer jumping (distance to ancestor, ancestor of ancestor)
    uint32_t anc[4], dep[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int i = kStart + lane + 64 * j;
        anc[j] = (uint32_t)nodeRoot;
        dep[j] = 0;
        if (i < nodeRoot) {
            anc[j] = hn[i].parent;
            dep[j] = 1;
        }
        L.tanc[lane + 64 * j] = (uint16_t)anc[j];
        L.tdep[lane + 64 * j] = (uint16_t)dep[j];
    }
    lds_sync();
    while (true) {
        bool more = false;
        uint32_t na[4], nd[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            na[j] = anc[j];
            nd[j] = dep[j];
            if (anc[j] != (uint32_t)nodeRoot) {
                nd[j] = dep[j] + L.tdep[anc[j] - kStart];
                na[j] = L.tanc[anc[j] - kStart];
                more |= na[j] != (uint32_t)nodeRoot;
            }
        }
        lds_sync();
#pragma unroll
        for (int j = 0; j < 4; j++) {
            anc[j] = na[j];
            dep[j] = nd[j];
            L.tanc[lane + 64 * j] = (uint16_t)na[j];
            L.tdep[lane + 64 * j] = (uint16_t)nd[j];
        }
        lds_sync();
        P.count(4);
        if (!ballot(more)) break;
    }
    // leaves: parent depth + 1
    uint32_t nbR[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int r = lane + 64 * j;
        nbR[j] = 0;
        if (r <= nonNullRank) {
            nbR[j] = (uint32_t)L.tdep[hn[r].parent - kStart] + 1u;
            hn[r].nbBits = (uint8_t)nbR[j];
        }
    }
    lds_sync();
    P.mark(12);
    // ---- HUF_setMaxHeight
    const uint32_t largestBits = hn[nonNullRank].nbBits;
    if (largestBits > maxNbBits) {
        const uint32_t baseCost = 1u << (largestBits - maxNbBits);
        int cost = 0;
        uint32_t nLess = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = lane + 64 * j;
            const bool in = r <= nonNullRank;
            if (in && nbR[j] > maxNbBits) {
                cost += (int)(baseCost - (1u << (largestBits - nbR[j])));
                nbR[j] = maxNbBits;
                hn[r].nbBits = (uint8_t)maxNbBits;
            }
            nLess += (uint32_t)__builtin_popcountll(ballot(in && nbR[j] < maxNbBits));
        }
        int totalCost = (int)wave_sum((uint32_t)cost);
        int n = (int)nLess - 1;  // last rank shorter than maxNbBits (depths grow with rank)
        totalCost >>= (largestBits - maxNbBits);
        const uint32_t noSymbol = 0xF0F0F0F0u;
        if (lane < 16) L.rankLast[lane] = noSymbol;
        lds_sync();
        // rankLast[maxNbBits - b] = last rank of length b (the reference's downward scan)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = lane + 64 * j;
            if (r <= n) {
                const uint32_t b = nbR[j];
                const uint32_t bn = (r == n) ? maxNbBits : (uint32_t)hn[r + 1].nbBits;
                if (b < bn) L.rankLast[maxNbBits - b] = (uint32_t)r;
            }
        }
        lds_sync();
        while (totalCost > 0) {
            unsigned nBitsToDecrease = z1::highbit32((uint32_t)totalCost) + 1;
            for (; nBitsToDecrease > 1; nBitsToDecrease--) {
                const uint32_t highPos = L.rankLast[nBitsToDecrease];
                const uint32_t lowPos = L.rankLast[nBitsToDecrease - 1];
                if (highPos == noSymbol) continue;
                if (lowPos == noSymbol) break;
                if (hn[highPos].count <= 2 * hn[lowPos].count) break;
            }
            while ((nBitsToDecrease <= z1::kHufTableLogMax) && (L.rankLast[nBitsToDecrease] == noSymbol)) nBitsToDecrease++;
            totalCost -= 1 << (nBitsToDecrease - 1);
            if (L.rankLast[nBitsToDecrease - 1] == noSymbol) L.rankLast[nBitsToDecrease - 1] = L.rankLast[nBitsToDecrease];
            const uint32_t rl = L.rankLast[nBitsToDecrease];
            hn[rl].nbBits = (uint8_t)(hn[rl].nbBits + 1);
            if (rl == 0) {
                L.rankLast[nBitsToDecrease] = noSymbol;
            } else {
                L.rankLast[nBitsToDecrease] = rl - 1;
                if (hn[rl - 1].nbBits != maxNbBits - nBitsToDecrease) L.rankLast[nBitsToDecrease] = noSymbol;
            }
            lds_sync();
        }
        while (totalCost < 0) {
            if (L.rankLast[1] == noSymbol) {
                while (hn[n].nbBits == maxNbBits) n--;
                hn[n + 1].nbBits = (uint8_t)(hn[n + 1].nbBits - 1);
                L.rankLast[1] = (uint32_t)(n + 1);
                totalCost++;
                lds_sync();
                continue;
            }
            const uint32_t rl = L.rankLast[1] + 1;
            hn[rl].nbBits = (uint8_t)(hn[rl].nbBits - 1);
            L.rankLast[1] = rl;
            totalCost++;
            lds_sync();
        }
        lds_sync();
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = lane + 64 * j;
            if (r <= nonNullRank) nbR[j] = hn[r].nbBits;
        }
    } else {
        maxNbBits = largestBits;
    }
    P.mark(13);
    // ---- canonical codes: starting value per length, then symbol order within a length
    {
        uint32_t mn = 0;
        for (int b = (int)maxNbBits; b > 0; b--) {
            uint32_t cnt = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) cnt += (uint32_t)__builtin_popcountll(ballot(nbR[j] == (uint32_t)b));
            if (lane == 0) L.vpr[b] = mn;
            mn = (mn + cnt) >> 1;
        }
        if (lane == 0) L.vpr[0] = 0;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int r = lane + 64 * j;
        if (r <= (int)maxSym) L.nbBits[hn[r].byte] = hn[r].nbBits;
    }
    lds_sync();
    uint32_t nbS[4], val[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t s = (uint32_t)lane + 64u * (uint32_t)j;
        nbS[j] = s <= maxSym ? L.nbBits[s] : 0xFFu;
        val[j] = 0;
    }
    for (uint32_t b = 0; b <= maxNbBits; b++) {
        uint32_t base = L.vpr[b];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t m = ballot(nbS[j] == b);
            if (nbS[j] == b) val[j] = base + mbcnt(m);
            base += (uint32_t)__builtin_popcountll(m);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t s = (uint32_t)lane + 64u * (uint32_t)j;
        if (s <= maxSym) L.val[s] = (uint16_t)val[j];
    }
    lds_sync();
    return maxNbBits;
}

// FSE_buildCTable_wksp for the weight alphabet (<= 13 symbols, tableLog <= 6, so a table entry per
// lane).  The serial spread visits positions (j * step) & mask for j = 0, 1, ... skipping those above
// highThreshold, and the k-th accepted visit takes the k-th slot of the symbols in order; the state
// table numbers each symbol's positions in increasing order (tableU16[cumul[s]++] = tableSize + u).
// Both are computed lane-parallel here (visit j / entry u in lane j / u, ranks by ballot): the serial
// loops were a chain of dependent LDS read-modify-writes, 64 per table.
__device__ __forceinline__ void fse_build_ctable_small(WCTable& ct, const int16_t* norm, unsigned maxSymbolValue,
                                                       unsigned tableLog, uint8_t* tableSymbol, uint32_t* cumul)
{
    (void)cumul;
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t tableMask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    ct.tableLog = tableLog;
    // symbol s in lane s: its count of positions (low-probability: 1) and the counts before it
    const int nv = (lane <= maxSymbolValue) ? (int)norm[lane] : 0;
    const bool low = nv == -1;
    const uint32_t cnt = low ? 1u : (nv > 0 ? (uint32_t)nv : 0u);
    const uint32_t excl = wave_incl_sum(cnt) - cnt;  // cumul[s]
    // low-probability symbols at the top, in symbol order
    const uint64_t lowMask = ballot(low);
    if (low) tableSymbol[tableSize - 1 - mbcnt(lowMask)] = (uint8_t)lane;
    const uint32_t highThreshold = tableSize - 1 - (uint32_t)__builtin_popcountll(lowMask);
    // the spread: the other symbols' slots
    const uint32_t ncnt = low ? 0u : cnt;
    const uint32_t nincl = wave_incl_sum(ncnt);  // slots of the symbols <= s
    const uint32_t pos = (lane * step) & tableMask;
    const bool valid = lane < tableSize && pos <= highThreshold;
    const uint32_t k = mbcnt(ballot(valid));  // this visit's slot
    uint32_t sym = 0;
    for (uint32_t q = 0; q <= maxSymbolValue; q++) sym += readlane_u32(nincl, (int)q) <= k ? 1u : 0u;
    if (valid) tableSymbol[pos] = (uint8_t)sym;
    lds_sync();
    // the state table: entry u's symbol, its rank among that symbol's entries, the symbol's cumul
    const bool isEntry = lane < tableSize;
    const uint32_t sy = isEntry ? tableSymbol[lane] : 0xFFu;
    uint32_t rank = 0;
    for (uint32_t q = 0; q <= maxSymbolValue; q++) {
        const uint64_t m = ballot(sy == q);
        if (sy == q) rank = mbcnt(m);
    }
    const uint32_t cs = (uint32_t)__shfl((int)excl, (int)(sy & 63u), 64);
    if (isEntry) ct.stateTable[cs + rank] = (uint16_t)(tableSize + lane);
    if (lane <= maxSymbolValue) {
        if (nv == 0) {
            ct.deltaNbBits[lane] = ((tableLog + 1) << 16) - (1u << tableLog);
            ct.deltaFindState[lane] = 0;
        } else if (nv == -1 || nv == 1) {
            ct.deltaNbBits[lane] = (tableLog << 16) - (1u << tableLog);
            ct.deltaFindState[lane] = (int32_t)excl - 1;
        } else {
            const uint32_t maxBitsOut = tableLog - z1::highbit32((uint32_t)(nv - 1));
            const uint32_t minStatePlus = (uint32_t)nv << maxBitsOut;
            ct.deltaNbBits[lane] = (maxBitsOut << 16) - minStatePlus;
            ct.deltaFindState[lane] = (int32_t)excl - nv;
        }
    }
    lds_sync();
}

__device__ __forceinline__ void wfse_init(uint32_t& st, const WCTable& ct, unsigned symbol)
{
    const uint32_t nbBitsOut = (ct.deltaNbBits[symbol] + (1u << 15)) >> 16;
    const uint32_t v = (nbBitsOut << 16) - ct.deltaNbBits[symbol];
    st = ct.stateTable[(v >> nbBitsOut) + ct.deltaFindState[symbol]];
}
__device__ __forceinline__ void wfse_encode(z1::BitW& bw, uint32_t& st, const WCTable& ct, unsigned symbol)
{
    const uint32_t nbBitsOut = (st + ct.deltaNbBits[symbol]) >> 16;
    z1::bw_add(bw, st, nbBitsOut);
    st = ct.stateTable[(st >> nbBitsOut) + ct.deltaFindState[symbol]];
}

// HUF_writeCTable into L.hdr from L.nbBits (wave-uniform; weights and their histogram by ballots).
// Returns the description size, 0 if it cannot be written (raw weights with > 128 symbols).
__device__ __noinline__ uint32_t huf_write_ctable_wave(uint32_t maxSym, uint32_t huffLog, PhaseProf& P)
{
    EncLds& L = sEnc;
    const int lane = lane_id();
    maxSym = uni(maxSym);
    huffLog = uni(huffLog);
    const uint32_t wtSize = maxSym;  // weights of symbols 0 .. maxSym-1
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t s = (uint32_t)lane + 64u * (uint32_t)j;
        w[j] = 0xFFu;
        if (s < wtSize) {
            const uint32_t nb = L.nbBits[s];
            w[j] = nb ? huffLog + 1 - nb : 0u;
            L.weights[s] = (uint8_t)w[j];
        }
    }
    for (uint32_t v = 0; v <= z1::kHufTableLogMax; v++) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) c += (uint32_t)__builtin_popcountll(ballot(w[j] == v));
        if (lane == 0) L.wcount[v] = c;
    }
    lds_sync();
    // HUF_compressWeights
    uint32_t hSize = 0;
    if (wtSize > 1) {
        unsigned maxW = z1::kHufTableLogMax;
        while (!L.wcount[maxW]) maxW--;
        uint32_t maxCount = 0;
        for (unsigned v = 0; v <= maxW; v++) maxCount = L.wcount[v] > maxCount ? L.wcount[v] : maxCount;
        if (maxCount == wtSize) {
            hSize = 1;
        } else if (maxCount > 1) {
            const unsigned tableLog = z1::fse_optimal_table_log(6, wtSize, maxW, 2);
            if (z1::fse_normalize(L.wnorm, tableLog, L.wcount, wtSize, maxW, false)) {
                lds_sync();
                const size_t nh = z1::fse_write_ncount(L.hdr + 1, L.wnorm, maxW, tableLog);
                if (nh && wtSize > 2) {
                    fse_build_ctable_small(L.fct, L.wnorm, maxW, tableLog, L.fscratch, L.wcumul);
                    // FSE_compress_usingCTable (two interleaved states) in two passes.  The states run
                    // serially and wave-uniform (table entry u / symbol s in lane u / s, read with
                    // v_readlane): chain X starts from the last weight, chain Y from the one before, and
                    // emission k (k = 0 .. n - 3) encodes weight n - 3 - k on chain X (k even) or Y (k
                    // odd); each emission only records its state and bit count into lane k & 63 of
                    // rec[k >> 6] (the reference's bit-container flushes do not change the bit order).
                    // Then the fields' offsets come from a wave prefix sum and their bits are ORed into
                    // the description in LDS, so the serial loop carries no bit packing (it was ~26
                    // scalar instructions per weight).
                    const uint32_t vST = ((uint32_t)lane < (1u << tableLog)) ? (uint32_t)L.fct.stateTable[lane] : 0u;
                    const uint32_t vDN = ((uint32_t)lane <= maxW) ? L.fct.deltaNbBits[lane] : 0u;
                    const uint32_t vDF = ((uint32_t)lane <= maxW) ? (uint32_t)L.fct.deltaFindState[lane] : 0u;
                    const uint32_t W4 = reinterpret_cast<const uint32_t*>(L.weights)[lane];
                    auto wsym = [&](uint32_t i) -> uint32_t {
                        return (readlane_u32(W4, (int)(i >> 2)) >> (8u * (i & 3u))) & 0xFFu;
                    };
                    auto init = [&](uint32_t sym) -> uint32_t {
                        const uint32_t dn = readlane_u32(vDN, (int)sym), df = readlane_u32(vDF, (int)sym);
                        const uint32_t nbo = (dn + (1u << 15)) >> 16;
                        const uint32_t v = (nbo << 16) - dn;
                        return readlane_u32(vST, (int)((v >> nbo) + df));
                    };
                    const uint32_t n = wtSize, nEm = n - 2;
                    // each emission's deltas, lane-parallel
                    uint32_t dnR[4], dfR[4], rec[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t k = (uint32_t)lane + 64u * (uint32_t)r;
                        const uint32_t sy = k < nEm ? (uint32_t)L.weights[n - 3 - k] : 0u;
                        dnR[r] = L.fct.deltaNbBits[sy];
                        dfR[r] = (uint32_t)L.fct.deltaFindState[sy];
                        rec[r] = 0;
                    }
                    uint32_t stX = init(wsym(n - 1)), stY = init(wsym(n - 2));
                    auto enc = [&](uint32_t& st, uint32_t& rc, uint32_t dv, uint32_t fv, uint32_t k) {
                        const uint32_t dn = readlane_u32(dv, (int)(k & 63u)), df = readlane_u32(fv, (int)(k & 63u));
                        const uint32_t nbo = (st + dn) >> 16;
                        // (one SGPR read per VALU instruction on gfx950: the lane select goes through m0)
                        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(rc) : "s"(st | (nbo << 16)), "{m0}"(k & 63u));
                        st = readlane_u32(vST, (int)((st >> nbo) + df));
                    };
#pragma unroll
                    for (uint32_t r = 0; r < 4; r++) {
                        const uint32_t kEnd = nEm < 64u * r + 64u ? nEm : 64u * r + 64u;
                        for (uint32_t k = 64u * r; k < kEnd; k += 2) {  // a pair never crosses a register
                            enc(stX, rec[r], dnR[r], dfR[r], k);
                            if (k + 1 < kEnd) enc(stY, rec[r], dnR[r], dfR[r], k + 1);
                        }
                    }
                    // FSE_flushCState of the second state, then the first (even n: X then Y; odd n: Y
                    // then X), then the end mark
                    const uint32_t fA = ((n & 1u) ? stY : stX) | (tableLog << 16), fB = ((n & 1u) ? stX : stY) | (tableLog << 16);
                    uint32_t pos[4], tot = 0;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t k = (uint32_t)lane + 64u * (uint32_t)r;
                        if (k == nEm) rec[r] = fA;
                        if (k == nEm + 1) rec[r] = fB;
                        if (k == nEm + 2) rec[r] = 1u | (1u << 16);
                        const uint32_t nb = k < nEm + 3 ? rec[r] >> 16 : 0u;
                        const uint32_t incl = wave_incl_sum(nb);
                        pos[r] = tot + incl - nb;
                        tot += readlane_u32(incl, 63);
                    }
                    const uint32_t bytes = (tot + 7) >> 3;
                    uint8_t* op = L.hdr + 1 + nh;
                    for (uint32_t b = (uint32_t)lane; b < bytes; b += 64) op[b] = 0;
                    lds_sync();
                    lds_u32* hw = (lds_u32*)(uint32_t*)L.hdr;  // 4-byte aligned (static_assert below)
                    const uint32_t B0 = 8u * (1u + (uint32_t)nh);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t k = (uint32_t)lane + 64u * (uint32_t)r;
                        if (k < nEm + 3) {
                            const uint32_t nb = rec[r] >> 16, v = rec[r] & ((1u << nb) - 1u);
                            const uint32_t P = B0 + pos[r], w = P >> 5, sh = P & 31u;
                            __hip_atomic_fetch_or(&hw[w], v << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            if (sh + nb > 32u)
                                __hip_atomic_fetch_or(&hw[w + 1], v >> (32u - sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                    }
                    hSize = (uint32_t)(nh + bytes);
                }
            }
        }
    }
    lds_sync();
    if (hSize > 1 && hSize < maxSym / 2) {
        if (lane == 0) L.hdr[0] = (uint8_t)hSize;
        lds_sync();
        return hSize + 1;
    }
    if (maxSym > 128) return 0;
    // raw 4-bit weights
    if (lane == 0) L.hdr[0] = (uint8_t)(128 + (maxSym - 1));
    if ((uint32_t)lane < (maxSym + 1) / 2) {
        const uint32_t a = L.weights[2 * lane], b = (2u * (uint32_t)lane + 1u < maxSym) ? L.weights[2 * lane + 1] : 0u;
        L.hdr[1 + lane] = (uint8_t)((a << 4) + b);
    }
    lds_sync();
    return (maxSym + 1) / 2 + 1;
}

// ---------------------------------------------------------------------------------------------
// Sequences section (ZSTD_compressSequences_internal, repeat mode none; zstd1_model.h
// compress_sequences): codes and their histograms in parallel over the sequences, table choice and
// FSE tables wave-uniform in LDS, then the serial backward encode over sequences staged 64 at a
// time into LDS.  Writes S.seqSection; returns its size, or (size_t)-1 / -2 for "emit a raw block".
// ---------------------------------------------------------------------------------------------
// FSE_buildCTable_wksp, wave-uniform, cumul / tableSymbol in LDS
__device__ __forceinline__ void fse_build_ctable_lds(z1::FseCTable& ct, const int16_t* norm, unsigned maxSymbolValue,
                                                     unsigned tableLog, uint8_t* tableSymbol, uint32_t* cumul)
{
    const uint32_t tableSize = 1u << tableLog;
    const uint32_t tableMask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
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
    uint32_t position = 0;
    for (unsigned symbol = 0; symbol <= maxSymbolValue; symbol++) {
        const int freq = norm[symbol];
        for (int k = 0; k < freq; k++) {
            tableSymbol[position] = (uint8_t)symbol;
            position = (position + step) & tableMask;
            while (position > highThreshold) position = (position + step) & tableMask;
        }
    }
    lds_sync();
    for (uint32_t u = 0; u < tableSize; u++) {
        const uint8_t sy = tableSymbol[u];
        const uint32_t cs = cumul[sy];
        ct.stateTable[cs] = (uint16_t)(tableSize + u);
        cumul[sy] = cs + 1;
    }
    unsigned total = 0;
    for (unsigned sy = 0; sy <= maxSymbolValue; sy++) {
        const int nv = norm[sy];
        if (nv == 0) {
            ct.deltaNbBits[sy] = ((tableLog + 1) << 16) - (1u << tableLog);
            ct.deltaFindState[sy] = 0;
        } else if (nv == -1 || nv == 1) {
            ct.deltaNbBits[sy] = (tableLog << 16) - (1u << tableLog);
            ct.deltaFindState[sy] = (int32_t)total - 1;
            total++;
        } else {
            const uint32_t maxBitsOut = tableLog - z1::highbit32((uint32_t)(nv - 1));
            const uint32_t minStatePlus = (uint32_t)nv << maxBitsOut;
            ct.deltaNbBits[sy] = (maxBitsOut << 16) - minStatePlus;
            ct.deltaFindState[sy] = (int32_t)total - nv;
            total += (unsigned)nv;
        }
    }
    lds_sync();
}

// little-endian bit writer into global memory, 32-bit flushes (byte-exact with z1::BitW)
struct GBitW {
    uint8_t* p;
    uint64_t acc;
    uint32_t n;
};
__device__ __forceinline__ void gbw_add(GBitW& b, uint32_t v, uint32_t nb)
{
    b.acc |= (uint64_t)(v & (uint32_t)((1ull << nb) - 1ull)) << b.n;
    b.n += nb;
    if (b.n >= 32) {
        if (lane_id() == 0) gst<uint32_t>(b.p, (uint32_t)b.acc);
        b.p += 4;
        b.acc >>= 32;
        b.n -= 32;
    }
}
__device__ __forceinline__ size_t gbw_close(GBitW& b, const uint8_t* start)
{
    gbw_add(b, 1, 1);
    const uint32_t nbytes = (b.n + 7) >> 3;
    if (lane_id() == 0)
        for (uint32_t i = 0; i < nbytes; i++) gst<uint8_t>(b.p + i, (uint8_t)(b.acc >> (8 * i)));
    return (size_t)(b.p + nbytes - start);
}
__device__ __forceinline__ void sfse_init(uint32_t& st, const z1::FseCTable& ct, unsigned symbol)
{
    const uint32_t nbBitsOut = (ct.deltaNbBits[symbol] + (1u << 15)) >> 16;
    const uint32_t v = (nbBitsOut << 16) - ct.deltaNbBits[symbol];
    st = ct.stateTable[(v >> nbBitsOut) + ct.deltaFindState[symbol]];
}
__device__ __forceinline__ void sfse_encode(GBitW& bw, uint32_t& st, const z1::FseCTable& ct, unsigned symbol)
{
    const uint32_t nbBitsOut = (st + ct.deltaNbBits[symbol]) >> 16;
    gbw_add(bw, st, nbBitsOut);
    st = ct.stateTable[(st >> nbBitsOut) + ct.deltaFindState[symbol]];
}

// the predefined LL / OF / ML compression tables (kSetBasic), built once per context
__device__ z1::FseCTable gSeqDefCT[3];
static_assert(sizeof(z1::FseCTable) % 4 == 0, "word copy");
__global__ __launch_bounds__(64) void seq_default_ctables_kernel()
{
    EncLds& L = sEnc;
    const int lane = lane_id();
#pragma unroll 1
    for (int k = 0; k < 3; k++) {
        const unsigned dmax = k == 0 ? z1::kMaxLL : (k == 1 ? z1::kDefaultMaxOff : z1::kMaxML);
        const unsigned lg = k == 0 ? z1::kLLDefaultNormLog : (k == 1 ? z1::kOFDefaultNormLog : z1::kMLDefaultNormLog);
        if ((unsigned)lane <= dmax)
            L.snorm[lane] = k == 0 ? z1::ll_default_norm(lane) : (k == 1 ? z1::of_default_norm(lane) : z1::ml_default_norm(lane));
        lds_sync();
        fse_build_ctable_lds(L.sct[k], L.snorm, dmax, lg, L.stsym, L.scumul);
        const uint32_t* w = (const uint32_t*)&L.sct[k];
        for (uint32_t u = (uint32_t)lane; u < sizeof(z1::FseCTable) / 4; u += 64) ((uint32_t*)&gSeqDefCT[k])[u] = w[u];
        lds_sync();
    }
}

__device__ __noinline__ size_t seq_section_wave(EncScratch S, uint32_t nbSeq)
{
    EncLds& L = sEnc;
    const uint32_t lane = (uint32_t)lane_id();
    nbSeq = uni(nbSeq);
    S.seqs = uni(S.seqs);
    S.codes = uni(S.codes);
    S.seqSection = uni(S.seqSection);
    S.maxSeq = uni(S.maxSeq);
    uint8_t* const dst = S.seqSection;
    uint8_t* llC = S.codes;
    uint8_t* ofC = S.codes + S.maxSeq;
    uint8_t* mlC = S.codes + 2 * S.maxSeq;
    const uint32_t* sq = (const uint32_t*)S.seqs;  // {litLength, offset, mlBase} per sequence
    // number of sequences
    uint32_t hl;
    if (nbSeq < 128) {
        if (lane == 0) gst<uint8_t>(dst, (uint8_t)nbSeq);
        hl = 1;
    } else if (nbSeq < 0x7F00) {
        if (lane == 0) { gst<uint8_t>(dst, (uint8_t)((nbSeq >> 8) + 0x80)); gst<uint8_t>(dst + 1, (uint8_t)nbSeq); }
        hl = 2;
    } else {
        if (lane == 0) { gst<uint8_t>(dst, 0xFF); gst<uint8_t>(dst + 1, (uint8_t)(nbSeq - 0x7F00)); gst<uint8_t>(dst + 2, (uint8_t)((nbSeq - 0x7F00) >> 8)); }
        hl = 3;
    }
    if (nbSeq == 0) return hl;
    uint8_t* const seqHead = dst + hl;
    uint8_t* op = seqHead + 1;
    // codes and histograms
    for (int k = 0; k < 3; k++) L.scount[k][lane] = 0;
    lds_sync();
    for (uint32_t i = lane; i < nbSeq; i += 64) {
        const uint32_t litLength = gld<uint32_t>(sq + 3 * i), offset = gld<uint32_t>(sq + 3 * i + 1),
                       mlBase = gld<uint32_t>(sq + 3 * i + 2);
        const uint32_t lc = z1::ll_code(litLength), oc = z1::highbit32(offset), mc = z1::ml_code(mlBase);
        gst<uint8_t>(llC + i, (uint8_t)lc);
        gst<uint8_t>(ofC + i, (uint8_t)oc);
        gst<uint8_t>(mlC + i, (uint8_t)mc);
        atomicAdd(&L.scount[0][lc], 1u);
        atomicAdd(&L.scount[1][oc], 1u);
        atomicAdd(&L.scount[2][mc], 1u);
    }
    lds_sync();
    const uint32_t last = nbSeq - 1;
    const uint32_t lastLL = gld<uint32_t>(sq + 3 * last), lastOff = gld<uint32_t>(sq + 3 * last + 1),
                   lastML = gld<uint32_t>(sq + 3 * last + 2);
    const uint32_t lastCode[3] = {z1::ll_code(lastLL), z1::highbit32(lastOff), z1::ml_code(lastML)};
    uint8_t* lastNCount = nullptr;
    uint32_t types[3];
    const unsigned maxes[3] = {z1::kMaxLL, z1::kMaxOff, z1::kMaxML};
    const unsigned fseLogs[3] = {z1::kLLFSELog, z1::kOffFSELog, z1::kMLFSELog};
    const unsigned normLogs[3] = {z1::kLLDefaultNormLog, z1::kOFDefaultNormLog, z1::kMLDefaultNormLog};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t cnt = (lane <= maxes[k]) ? L.scount[k][lane] : 0u;
        const uint64_t nz = ballot(cnt != 0);
        const unsigned mx = 63u - (unsigned)__builtin_clzll(nz);
        const uint32_t mostFrequent = wave_max(cnt);
        const bool defaultAllowed = (k == 1) ? (mx <= z1::kDefaultMaxOff) : true;
        const unsigned type = z1::select_encoding_type(mostFrequent, nbSeq, normLogs[k], defaultAllowed);
        types[k] = type;
        z1::FseCTable& ct = L.sct[k];
        if (type == z1::kSetRle) {
            ct.tableLog = 0;
            ct.stateTable[0] = 0;
            ct.stateTable[1] = 0;
            ct.deltaNbBits[mx] = 0;
            ct.deltaFindState[mx] = 0;
            if (lane == 0) gst<uint8_t>(op, (uint8_t)lastCode[k]);
            op += 1;
        } else if (type == z1::kSetBasic) {  // the predefined table, built once (seq_default_ctables_kernel)
            const uint32_t* w = (const uint32_t*)&gSeqDefCT[k];
            for (uint32_t u = lane; u < sizeof(z1::FseCTable) / 4; u += 64) ((uint32_t*)&ct)[u] = gld<uint32_t>(w + u);
        } else {
            size_t nbSeq_1 = nbSeq;
            const unsigned tableLog = z1::fse_optimal_table_log(fseLogs[k], nbSeq, mx, 2);
            if (L.scount[k][lastCode[k]] > 1) {
                L.scount[k][lastCode[k]] -= 1;
                nbSeq_1--;
            }
            lds_sync();
            if (!z1::fse_normalize(L.snorm, tableLog, L.scount[k], nbSeq_1, mx, nbSeq_1 >= 2048)) return (size_t)-2;
            lds_sync();
            const size_t nc = z1::fse_write_ncount(L.snc, L.snorm, mx, tableLog);
            if (nc == 0) return (size_t)-2;
            lds_sync();
            for (uint32_t i = lane; i < nc; i += 64) gst<uint8_t>(op + i, L.snc[i]);
            fse_build_ctable_lds(ct, L.snorm, mx, tableLog, L.stsym, L.scumul);
            lastNCount = op;
            op += nc;
        }
        lds_sync();
    }
    if (lane == 0) gst<uint8_t>(seqHead, (uint8_t)((types[0] << 6) + (types[1] << 4) + (types[2] << 2)));
    // ZSTD_encodeSequences (no long offsets: windowLog <= 17), backwards
    GBitW bw{op, 0, 0};
    uint32_t sLL, sOF, sML;
    sfse_init(sML, L.sct[2], lastCode[2]);
    sfse_init(sOF, L.sct[1], lastCode[1]);
    sfse_init(sLL, L.sct[0], lastCode[0]);
    gbw_add(bw, lastLL, z1::ll_bits(lastCode[0]));
    gbw_add(bw, lastML, z1::ml_bits(lastCode[2]));
    gbw_add(bw, lastOff, lastCode[1]);
    for (int32_t blk = (int32_t)(last - 1) >> 6; blk >= 0 && last > 0; blk--) {
        const uint32_t i = 64u * (uint32_t)blk + lane;
        lds_sync();
        if (i < last) {
            L.sv[0][lane] = gld<uint32_t>(sq + 3 * i);
            L.sv[1][lane] = gld<uint32_t>(sq + 3 * i + 2);
            L.sv[2][lane] = gld<uint32_t>(sq + 3 * i + 1);
            L.sc[0][lane] = gb(llC + i);
            L.sc[1][lane] = gb(ofC + i);
            L.sc[2][lane] = gb(mlC + i);
        }
        lds_sync();
        const int32_t top = (64 * blk + 63 < (int32_t)last - 1) ? 63 : (int32_t)last - 1 - 64 * blk;
        for (int32_t t = top; t >= 0; t--) {
            const uint32_t lc = L.sc[0][t], oc = L.sc[1][t], mc = L.sc[2][t];
            sfse_encode(bw, sOF, L.sct[1], oc);
            sfse_encode(bw, sML, L.sct[2], mc);
            sfse_encode(bw, sLL, L.sct[0], lc);
            gbw_add(bw, L.sv[0][t], z1::ll_bits(lc));
            gbw_add(bw, L.sv[1][t], z1::ml_bits(mc));
            gbw_add(bw, L.sv[2][t], oc);
        }
    }
    gbw_add(bw, sML, L.sct[2].tableLog);
    gbw_add(bw, sOF, L.sct[1].tableLog);
    gbw_add(bw, sLL, L.sct[0].tableLog);
    const size_t streamSize = gbw_close(bw, op);
    op += streamSize;
    if (lastNCount && (op - lastNCount) < 4) return (size_t)-1;
    return (size_t)(op - dst);
}

// ---------------------------------------------------------------------------------------------
// Literals section (ZSTD_compressLiterals).  Writes at dst, returns its size.
// ---------------------------------------------------------------------------------------------
__device__ inline size_t write_raw_literals_wave(uint8_t* dst, const uint8_t* lit, uint32_t n)
{
    size_t fl = z1::raw_lit_header_size(n);
    if (lane_id() == 0) z1::write_rawrle_lit_header(dst, n, z1::kSetBasic);
    wave_copy(dst + fl, lit, n);
    return fl + n;
}

// writeRaw = false: a raw literals section is sized but not written (the caller knows it turns the
// whole block raw and writes that instead).
// Huffman table state of the frame (zstd1_model.h compress_literals): prevCw holds the confirmed
// table of an earlier block (code | nbBits << 16 per symbol) when prevCheck (HUF_repeat_check); a
// newly built table is written to nextCw when saveNew (a later block may repeat it).
struct LitOut {
    uint32_t size;
    uint32_t newTable;  // a new table was built and used (HUF_repeat_check from here on)
};
template <bool COOP>
__device__ __noinline__ LitOut compress_literals_wave(uint8_t* __restrict__ dst, const uint8_t* __restrict__ lit, uint32_t n,
                                                      PhaseProf& P, uint32_t writeRaw, const uint32_t* prevCw,
                                                      uint32_t prevCheck, uint32_t* nextCw, uint32_t saveNew,
                                                      uint32_t rawAt, lds_enc_cmd* coop)
{
    EncLds& L = sEnc;
    dst = uni(dst);
    lit = uni(lit);
    n = uni(n);
    writeRaw = uni(writeRaw);
    prevCw = uni(prevCw);
    prevCheck = uni(prevCheck);
    nextCw = uni(nextCw);
    saveNew = uni(saveNew);
    rawAt = uni(rawAt);  // a section of this size or more makes the block raw: it is then only sized
    auto ret = [](size_t sz, bool nt) { LitOut o; o.size = (uint32_t)sz; o.newTable = nt ? 1u : 0u; return o; };
    auto write_raw_literals_wave = [&](uint8_t* d, const uint8_t* l, uint32_t m) -> size_t {
        if (writeRaw) return pgn::write_raw_literals_wave(d, l, m);
        return z1::raw_lit_header_size(m) + m;
    };
    const int lane = lane_id();
    if (n <= 63) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
    const uint32_t minGain = (n >> 6) + 2;
    const uint32_t lhSize = (uint32_t)z1::huf_lit_header_size(n);
    const bool single = n < 256;
    const uint32_t segSize = single ? n : (n + 3) / 4;
    const int nseg = single ? 1 : 4;
    for (int i = lane; i < 2 * 256; i += 64) {
        (&L.hist2[0][0])[i] = 0;
        L.hist2x[1 + i] = 0;
    }
    wave_sync();
    if (COOP && !single) {  // the four segments' histograms on the four waves
        if (lane == 0) {
            coop->op = 1;
            coop->lit = lit;
            coop->n = n;
            coop->segSize = segSize;
        }
        __syncthreads();  // B1
        hist_segment_wave(lit, n, segSize, 0);
        __syncthreads();  // B2
    }
    // per-segment histograms; the 16-byte loads of four 1024-byte steps are issued together.  A
    // block's segment i / segSize is one multiply-high by ceil(2^32 / segSize): exact here because
    // i < 2^17 (a block is at most 128 KiB) and segSize <= 2^15, so i times the reciprocal's error
    // stays below 2^32 (the general division took ~15 instructions per block)
    const uint32_t segMagic = 0xFFFFFFFFu / segSize + 1u;
    for (uint32_t i0 = (uint32_t)lane * 16; i0 < ((COOP && !single) ? 0u : n); i0 += 4096) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 1024u * (uint32_t)u;
            if (i + 16 <= n) {
                v[u] = gld<uint4>(lit + i);
            } else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (uint32_t k = 0; k < 16; k++)
                    if (i + k < n) w[k >> 2] |= (uint32_t)gb(lit + i + k) << (8 * (k & 3));
                v[u] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 1024u * (uint32_t)u;
            const uint32_t wd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            const uint32_t sa = __umulhi(i, segMagic);
            const uint32_t boundary = (sa + 1) * segSize;
            if (i + 16 <= n && i + 16 <= boundary) {  // the usual case: 16 bytes of one segment
                uint32_t* h = ((lane & 1) ? &L.hist2x[1] : &L.hist2[0][0]) + 256 * (sa >> 1);
                const uint32_t inc = 1u << (16 * (sa & 1));
#pragma unroll
                for (int k = 0; k < 16; k++) atomicAdd(h + ((wd[k >> 2] >> (8 * (k & 3))) & 0xFFu), inc);
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    if (i + k < n) {
                        const uint32_t sg = (i + k < boundary) ? sa : sa + 1;
                        atomicAdd(&L.hist2[sg >> 1][(wd[k >> 2] >> (8 * (k & 3))) & 0xFFu], 1u << (16 * (sg & 1)));
                    }
                }
            }
        }
    }
    wave_sync();
    P.count(8, (n + 4095) / 4096);
    uint32_t c[4];
    uint32_t myMaxSym = 0, myLargest = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int s = lane + 64 * q;
        const uint32_t h01 = L.hist2[0][s] + L.hist2x[1 + s], h23 = L.hist2[1][s] + L.hist2x[1 + 256 + s];
        L.hist2[0][s] = h01;
        L.hist2[1][s] = h23;
        c[q] = (h01 & 0xFFFFu) + (h01 >> 16) + (h23 & 0xFFFFu) + (h23 >> 16);
        L.count[s] = c[q];
        if (c[q]) myMaxSym = (uint32_t)s;
        myLargest = c[q] > myLargest ? c[q] : myLargest;
    }
    const uint32_t maxSym = wave_max(myMaxSym);
    const uint32_t largest = wave_max(myLargest);
    wave_sync();
    P.mark(3);
#if PGN_AB_SKIP == 3
    { size_t r = write_raw_literals_wave(dst, lit, n); return ret(r, false); }
#endif
    if (largest == n) {  // one symbol: RLE literals
        size_t fl = z1::raw_lit_header_size(n);
        if (lane == 0) {
            z1::write_rawrle_lit_header(dst, n, z1::kSetRle);
            dst[fl] = lit[0];
        }
        return ret(fl + 1, false);
    }
    if (largest <= (n >> 7) + 4) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
    // HUF_validateCTable: the previous table must code every symbol present; a valid one is kept
    // for small inputs (preferRepeat) or when it is estimated no worse than a new table + its header
    uint32_t oldNb[4] = {0, 0, 0, 0};
    bool repeat = false;
    if (prevCheck) {
        bool bad = false;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            oldNb[q] = gld<uint32_t>(prevCw + lane + 64 * q) >> 16;
            bad |= c[q] != 0 && oldNb[q] == 0;
        }
        repeat = !ballot(bad);
    }
    bool useOld = repeat && n <= 1024;
    uint32_t hSize = 0;
    if (!useOld) {
    unsigned huffLog = z1::huf_optimal_table_log(z1::kHufTableLogDefault, n, maxSym);
    // HUF_sort: rank = #greater + #equal-with-smaller-symbol (stable, decreasing count)
    for (int i = lane; i < 2 * 256 + 4; i += 64) {
        L.nodes[i].count = 0; L.nodes[i].parent = 0; L.nodes[i].byte = 0; L.nodes[i].nbBits = 0;
    }
    wave_sync();
    {
        // HUF_sort order = descending key count << 8 | (255 - symbol) (stable by symbol): a bitonic
        // sort of the 256 keys, four per lane (element e = lane + 64q), ascending on ~key so that
        // absent symbols (key 0) come last; sorted element e is then the leaf of rank e
        uint32_t a[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t sy = (uint32_t)lane + 64u * (uint32_t)q;
            a[q] = (sy <= maxSym) ? ~((c[q] << 8) | (255u - sy)) : 0xFFFFFFFFu;
        }
#pragma unroll
        for (uint32_t k = 2; k <= 256; k <<= 1) {
#pragma unroll
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                if (j >= 64) {  // partner in another register of the same lane
                    const uint32_t qj = j >> 6;
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++) {
                        if (q & qj) continue;
                        const uint32_t q2 = q | qj;
                        const uint32_t mn = a[q] < a[q2] ? a[q] : a[q2], mx = a[q] < a[q2] ? a[q2] : a[q];
                        const bool asc = ((64u * q) & k) == 0;
                        a[q] = asc ? mn : mx;
                        a[q2] = asc ? mx : mn;
                    }
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++) {
                        const uint32_t b = (uint32_t)__shfl_xor((int)a[q], (int)j, 64);
                        const uint32_t mn = a[q] < b ? a[q] : b, mx = a[q] < b ? b : a[q];
                        const uint32_t e = (uint32_t)lane + 64u * q;
                        const bool lower = (e & j) == 0, asc = (e & k) == 0;
                        a[q] = (lower == asc) ? mn : mx;
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t r = (uint32_t)lane + 64u * (uint32_t)q;
            if (r <= maxSym) {
                const uint32_t key = ~a[q];
                L.nodes[1 + r].count = key >> 8;
                L.nodes[1 + r].byte = (uint8_t)(255u - (key & 0xFFu));
            }
        }
    }
    wave_sync();
    P.mark(4);
    uint32_t nnz = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) nnz += (uint32_t)__builtin_popcountll(ballot(c[q] != 0));
    const uint32_t hl = huf_tree_wave(maxSym, huffLog, nnz, P);
    P.mark(14);
#if PGN_AB_SKIP == 5  // diagnostic: stop after the tree (instruction attribution of the table description)
    { size_t r = write_raw_literals_wave(dst, lit, n); return ret(r + 0 * hl, false); }
#endif
    if (!repeat) {
        // the streams alone already miss the gain the section must make: raw literals whatever the
        // table description's size (HUF_compress_internal's final check), so it is not written
        uint32_t b4[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int s = lane + 64 * q;
            const uint32_t nbq = ((uint32_t)s <= maxSym) ? (uint32_t)L.nbBits[s] : 0u;
#pragma unroll
            for (int k = 0; k < 4; k++) b4[k] += seg_count(L, k, s) * nbq;
        }
        uint32_t cs = single ? 0u : 6u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k == 0 || !single) cs += (wave_sum(b4[k]) + 8) >> 3;
        if (cs >= n - minGain) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
        if (lhSize + cs >= rawAt) { P.mark(7); return ret(lhSize + cs, false); }
    }
    hSize = huf_write_ctable_wave(maxSym, hl, P);
    P.count(5);
    P.count(6, maxSym);
    P.mark(5);
    if (hSize == 0) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
    if (repeat) {  // HUF_estimateCompressedSize of the old and the new table
        uint32_t eo = 0, en = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int s = lane + 64 * q;
            eo += c[q] * oldNb[q];
            en += c[q] * (((uint32_t)s <= maxSym) ? (uint32_t)L.nbBits[s] : 0u);
        }
        const uint32_t oldSize = wave_sum(eo) >> 3, newSize = wave_sum(en) >> 3;
        useOld = oldSize <= hSize + newSize || hSize + 12 >= n;
    }
    if (!useOld && hSize + 12 >= n) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
    }  // !useOld
    if (useOld) hSize = 0;  // a repeated table has no description
    // exact stream sizes from the segment histograms
    uint32_t bytes[4] = {0, 0, 0, 0}, bits[4] = {0, 0, 0, 0};
    {
        uint32_t b4[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int s = lane + 64 * q;
            uint32_t cwq;
            if (useOld) cwq = gld<uint32_t>(prevCw + s);
            else cwq = ((uint32_t)s <= maxSym) ? ((uint32_t)L.val[s] | ((uint32_t)L.nbBits[s] << 16)) : 0u;
            L.cw[s] = cwq;
            const uint32_t nbq = cwq >> 16;
#pragma unroll
            for (int k = 0; k < 4; k++) b4[k] += seg_count(L, k, s) * nbq;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            bits[k] = wave_sum(b4[k]);
            bytes[k] = (bits[k] + 8) >> 3;
        }
    }
    uint32_t cStreams = single ? bytes[0] : 6 + bytes[0] + bytes[1] + bytes[2] + bytes[3];
    uint32_t total = hSize + cStreams;
    if (total >= n - 1 || total >= n - minGain) { size_t r = write_raw_literals_wave(dst, lit, n); P.mark(7); return ret(r, false); }
    if (lhSize + total >= rawAt) { P.mark(7); return ret(lhSize + total, false); }
    if (!useOld && saveNew) {  // the table a later block may repeat
#pragma unroll
        for (int q = 0; q < 4; q++) gst<uint32_t>(nextCw + lane + 64 * q, L.cw[lane + 64 * q]);
    }
    if (lane == 0) {
        z1::write_huf_lit_header(dst, lhSize, n, total, single, useOld ? z1::kSetRepeat : z1::kSetCompressed);
        if (!single) {
            z1::wr16(dst + lhSize + hSize, bytes[0]);
            z1::wr16(dst + lhSize + hSize + 2, bytes[1]);
            z1::wr16(dst + lhSize + hSize + 4, bytes[2]);
        }
    }
    for (uint32_t i = (uint32_t)lane; i < hSize; i += 64) gst<uint8_t>(dst + lhSize + i, L.hdr[i]);
    wave_sync();
    uint8_t* op = dst + lhSize + hSize + (single ? 0 : 6);
    if (COOP && !single) {  // the four segments' bit packing on the four waves
        if (lane == 0) {
            coop->op = 2;
            coop->lit = lit;
            coop->n = n;
            coop->segSize = segSize;
            uint8_t* o = op;
            for (int k = 0; k < 4; k++) {
                coop->out[k] = o;
                coop->bits[k] = bits[k];
                o += bytes[k];
            }
        }
        __syncthreads();  // B1
        huf_encode_segment_wave(op, lit, segSize, bits[0], (lds_u32*)sEnc.win);
        __syncthreads();  // B2
    } else {
        for (int k = 0; k < nseg; k++) {
            uint32_t a = segSize * (uint32_t)k;
            uint32_t e = (k == nseg - 1) ? n : a + segSize;
#if PGN_AB_SKIP != 4
            huf_encode_segment_wave(op, lit + a, e - a, bits[k], (lds_u32*)sEnc.win);
#endif
            P.count(7, (e - a + 1023) / 1024);
            op += bytes[k];
        }
    }
    P.mark(6);
    return ret(lhSize + total, !useOld);
}

// ---------------------------------------------------------------------------------------------
// One stream -> one frame of up to kMaxFrameBytes (ZSTD_compress_frameChunk: blocks of 128 KiB;
// the block logic and the state a frame carries across its blocks -- hash table, repeat offsets,
// Huffman table -- are zstd1_model.h compress_block).  dst must have compress_bound(n) bytes.
// Returns the frame size.
// ---------------------------------------------------------------------------------------------
__device__ inline bool wave_is_rle(const uint8_t* p, uint32_t n)  // ZSTD_isRLE
{
    const uint8_t b0 = gb(p);
    bool diff = false;
    for (uint32_t i = (uint32_t)lane_id(); i < n; i += 64) diff |= gb(p + i) != b0;
    return !ballot(diff);
}

template <bool COOP = false>
__device__ __noinline__ size_t zstd1_compress_wave(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n,
                                             EncScratch S, uint32_t tag, PhaseProf& P)
{
    dst = uni(dst);
    src = uni(src);
    n = uni(n);
    tag = uni(tag);
    S.ht = uni(S.ht);
    S.seqs = uni(S.seqs);
    S.codes = uni(S.codes);
    S.lit = uni(S.lit);
    S.seqSection = uni(S.seqSection);
    S.seqWork = uni(S.seqWork);
    S.maxSeq = uni(S.maxSeq);
    S.huf = uni(S.huf);
    const int lane = lane_id();
    if (n == 0) {
        if (lane == 0) z1::write_empty_frame(dst);
        return 9;
    }
    const size_t h = z1::frame_header_size(n, n < 7 ? 10u : z1::level1_params(n).windowLog);
    if (n < 7) {
        if (lane == 0) z1::write_raw_block_frame(dst, src, n);
        return h + 3 + n;
    }
    const z1::Params p = z1::level1_params(n);
    P.count(12);
    if (lane == 0) z1::write_frame_header(dst, n, p.windowLog);
    size_t o = h;
    uint32_t rep0 = 1, rep1 = 4;  // confirmed repeat offsets (rep[2] is never read at level 1)
    uint32_t hufCur = 0, hufCheck = 0;
    for (uint32_t start = 0; start < n; start += (uint32_t)z1::kMaxSrc) {
        const uint32_t bs = (n - start < (uint32_t)z1::kMaxSrc) ? n - start : (uint32_t)z1::kMaxSrc;
        const bool last = start + bs == n, first = start == 0;
        uint8_t* bdst = dst + o;
        uint32_t cSize = 0;  // 0: raw block, 1: RLE block, else compressed body size
        size_t seqSize = 0;
#if PGN_AB_SKIP == 1
        if (false) {
#else
        if (bs >= 7) {
#endif
            const uint32_t ip0 = start + (start == 0 ? 1u : 0u);
            const SearchOut so = fast_search_wave(src, start, start + bs, p.hashLog, p.mls, S.ht, tag, S.seqs, rep0, rep1,
                                                  ht_idx_bits(n), z1::window_low_index(start + bs, p.windowLog),
                                                  ip0 + 1u - z1::window_low_index(ip0, p.windowLog), first && last);
            const uint32_t nbSeq = uni(so.nbSeq), lastLL = uni(so.lastLL);
            P.mark(1);
            P.count(0, uni(so.rounds));
            P.count(14, uni(so.candIters));
            P.count(1, nbSeq);
            P.count(13);
#if PGN_AB_SKIP == 2
            if (uni(so.nbSeq) < 0x7FFFFFFFu) goto raw_block;
#endif
            const uint8_t* lit = src + start;
            uint32_t nLit = bs;
            if (nbSeq > 0) {
                // gather the literal runs
                uint32_t pos = start, q = 0;
                for (uint32_t i = 0; i < nbSeq; i++) {
                    const z1::Seq sq = S.seqs[i];
                    wave_copy(S.lit + q, src + pos, sq.litLength);
                    q += sq.litLength;
                    pos += sq.litLength + sq.mlBase + 3;
                }
                wave_copy(S.lit + q, src + pos, lastLL);
                q += lastLL;
                wave_sync();
                lit = S.lit;
                nLit = q;
                P.mark(2);
            }
            uint8_t* body = bdst + 3;
            // without sequences a raw literals section makes the block raw (lh + n + 1 >= maxCSize): it
            // is then only sized here, and the raw block below is the one copy
            // without sequences the block is compressed only if litSize + 1 < maxCSize
            const uint32_t maxCSize = bs - ((bs >> 6) + 2);
            const LitOut lo = compress_literals_wave<COOP>(body, lit, nLit, P, nbSeq > 0 ? 1u : 0u, S.huf + 256 * hufCur,
                                                           hufCheck, S.huf + 256 * (hufCur ^ 1u), last ? 0u : 1u,
                                                           nbSeq == 0 ? maxCSize - 1u : 0xFFFFFFFFu, S.coop);
            const size_t litSize = uni(lo.size);
            wave_sync();
            if (nbSeq == 0) {
                if (lane == 0) body[litSize] = 0;
                seqSize = 1;
            } else {
                P.count(10);
                P.count(11, nbSeq);
                const size_t r = seq_section_wave(S, nbSeq);
                seqSize = (r == (size_t)-1 || r == (size_t)-2) ? (size_t)-1 : r;
                P.mark(8);
            }
            if (seqSize != (size_t)-1 && litSize + seqSize < maxCSize) cSize = (uint32_t)(litSize + seqSize);
            // a later block of one repeated byte is an RLE block (never the first: decoders <= 1.4.3)
            if (!first && cSize < 25 && wave_is_rle(src + start, bs)) cSize = 1;
            if (cSize > 1) {  // ZSTD_confirmRepcodesAndEntropyTables
                rep0 = uni(so.rep0);
                rep1 = uni(so.rep1);
                if (uni(lo.newTable)) {
                    hufCur ^= 1u;
                    hufCheck = 1;
                }
            }
        }
#if PGN_AB_SKIP == 2
    raw_block:
#endif
        wave_sync();
        size_t bsz;
        if (cSize == 0) {
            if (lane == 0) z1::wr24(bdst, (uint32_t)((last ? 1u : 0u) + (z1::kBtRaw << 1) + (bs << 3)));
            wave_copy_nt(bdst + 3, src + start, bs);  // into the blob once: non-temporal
            bsz = 3 + bs;
        } else if (cSize == 1) {
            if (lane == 0) {
                z1::wr24(bdst, (uint32_t)((last ? 1u : 0u) + (z1::kBtRle << 1) + (bs << 3)));
                bdst[3] = src[start];
            }
            bsz = 4;
        } else {
            if (seqSize > 1) wave_copy(bdst + 3 + (cSize - seqSize), S.seqSection, seqSize);
            if (lane == 0) z1::wr24(bdst, (uint32_t)((last ? 1u : 0u) + (z1::kBtCompressed << 1) + (cSize << 3)));
            bsz = 3 + cSize;
        }
        o += bsz;
        wave_sync();
        P.mark(9);
    }
    return o;
}

}  // namespace pgn
