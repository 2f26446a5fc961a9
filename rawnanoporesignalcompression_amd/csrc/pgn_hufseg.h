// pgn_hufseg.h -- the four Huffman streams of a zstd literals section (HUF_decompress4X1: the literal
// stage of every ZSTD_decompress call at C5.hpp:588-667 and signal_compression.cpp:112-118), decoded
// by one wave in ONE pass.  Included by pgn_zdec.h after the decoder's LDS (sDec) is declared.
//
// Each stream is cut into S <= 16 segments of equal bit length, one lane per segment (lanes 16k..16k+S-1
// decode stream k).  Lane j > 0 starts kSegOv bits above its segment's top (speculatively: the true
// codeword grid is unknown there), decodes without output down to the top, then outputs every symbol
// down to its segment's bottom, recording the codeword starts of its first kSegRec bits in a bitmap.
// A Huffman decoder resynchronises within a few codewords, so by the segment top the speculative path
// has almost always joined the true one.  Afterwards lane j checks its exit (the first true codeword
// start at or below its bottom: on the true path, because lane j-1 checked its own) against lane
// j+1's bitmap: a recorded start means lane j+1's symbols from there on are the true ones (the few
// above it are dropped); an unrecorded one makes lane j decode on ("walk") until it meets one.  If
// the walk leaves lane j+1's recorded bits, lane j stops there and lane j+1 decodes its segment again
// from that (true) position, then syncs with lane j+2 in turn ("epochs"); a stream whose segments
// never meet (e.g. a code of equal lengths cut off its grid) is thus decoded lane after lane, never
// wrongly.
//
// The stream's bits reach the lanes in wave-uniform ROUNDS: each lane's 16-word window of the stream
// is staged into LDS (word-major, sDec.stg[w & 15][lane]) from registers loaded one round earlier, and
// in a round a lane decodes until its position nears the window's bottom (kSegStride words a round).
// Bodies of four symbols leave as one dword store.  Every segment writes into its own region of a
// scratch area; the valid range of every region is finally copied to the stream's place in the
// destination ("compaction").  Every symbol is decoded once (plus the overlaps and the rare walks).
#pragma once

namespace pgn {

constexpr int kSegMax = 16;              // segments (lanes) per stream
constexpr int32_t kSegOv = 128;          // speculative overlap decoded above a segment's top
constexpr int32_t kSegRec = 128;         // codeword starts recorded below a segment's top (sync window)
constexpr int32_t kSegMinBits = 1536;    // shortest segment worth a lane of its own
constexpr int32_t kSegStride = 8;        // window words consumed per round (the half that is restaged)
constexpr int kSegMaxEpochs = kSegMax + 2;

// ---------------------------------------------------------------------------------------------
// Per-lane backward bit reader.  Positions are bit offsets from `base` (a 16-byte aligned address at
// or below the stream's first byte); the stream occupies bytes [off, end) of base.  W holds bits
// [wlo, wlo + 64), nx the word below it; the lane's window (staged words [wb, wb + 16)) serves the
// refills.
// ---------------------------------------------------------------------------------------------
struct SegRd {
    const uint8_t* base;
    int32_t off, end;
    uint64_t W;
    int32_t wlo;
    uint32_t nx;
    int32_t wb;
};

// words [w, w + 4) of base (w % 4 == 0: one aligned 16-byte piece), bytes outside the stream
// [off, end) read as zero.  A piece that holds any stream byte is loaded whole (it lies in the same
// 16-byte block, so in the same page, as that byte) and the outside bytes are masked off; a piece
// with none is not loaded.  Branch-free, so the prefetch of a round never waits on anything.
__device__ __forceinline__ uint32_t seg_keep(int32_t lo, int32_t hi, int32_t i)  // bytes [lo, hi) of dword i
{
    const int32_t a = lo - 4 * i, z = hi - 4 * i;  // keep bytes a .. z-1 of this dword
    const uint32_t ma = a <= 0 ? ~0u : (a >= 4 ? 0u : (~0u << (8 * a)));
    const uint32_t mz = z >= 4 ? ~0u : (z <= 0 ? 0u : (~0u >> (32 - 8 * z)));
    return ma & mz;
}
__device__ __forceinline__ uint4 seg_load4(const SegRd& r, int32_t w)
{
    const int32_t b = 4 * w;
    if (b + 16 <= r.off || b >= r.end) return make_uint4(0u, 0u, 0u, 0u);
    uint4 v = gld<uint4>(r.base + b);
    if (b < r.off || b + 16 > r.end) {
        const int32_t lo = r.off - b, hi = r.end - b;
        v.x &= seg_keep(lo, hi, 0);
        v.y &= seg_keep(lo, hi, 1);
        v.z &= seg_keep(lo, hi, 2);
        v.w &= seg_keep(lo, hi, 3);
    }
    return v;
}
// the prefetch form: pieces wholly inside or outside the stream only; a piece across the stream's
// first byte (once per lane and stream) is left to seg_load4 at staging time (*edge set), so that no
// wait follows the prefetch's loads
__device__ __forceinline__ uint4 seg_prefetch4(const SegRd& r, int32_t w, bool& edge)
{
    const int32_t b = 4 * w;
    const bool out = b + 16 <= r.off || b >= r.end, in = b >= r.off && b + 16 <= r.end;
    edge = !out && !in;
    return in ? gld<uint4>(r.base + b) : make_uint4(0u, 0u, 0u, 0u);
}
// words [w, w + 4) into the lane's ring column (slots w & 15 .. (w + 3) & 15; w % 4 == 0)
__device__ __forceinline__ void seg_put4(int32_t w, const uint4& v, int lane)
{
    sDec.stg[w & 15][lane] = v.x;
    sDec.stg[(w + 1) & 15][lane] = v.y;
    sDec.stg[(w + 2) & 15][lane] = v.z;
    sDec.stg[(w + 3) & 15][lane] = v.w;
}
// the first window of a reader at P: 4-word aligned, words P/32 - 15 .. P/32 at least
__device__ __forceinline__ int32_t seg_first_wb(int32_t P) { return ((P >> 5) - 12) & ~3; }
// the whole window [wb, wb + 16), loaded and staged at once (first round, walks, restarts)
__device__ __forceinline__ void seg_stage_full(const SegRd& r, int32_t wb, int lane)
{
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = seg_load4(r, wb + 4 * i);
#pragma unroll
    for (int i = 0; i < 4; i++) seg_put4(wb + 4 * i, v[i], lane);
}
// reader at P from the staged window: W = words (P/32 - 1, P/32)
__device__ __forceinline__ void seg_attach(SegRd& r, int32_t P, int lane)
{
    const int32_t cur = (P >> 5) - 1;
    r.wlo = 32 * cur;
    r.W = (uint64_t)sDec.stg[cur & 15][lane] | ((uint64_t)sDec.stg[(cur + 1) & 15][lane] << 32);
    r.nx = sDec.stg[(cur - 1) & 15][lane];
}
// two table entries: the codeword at P and the one below it (refill first: P - wlo >= 2 tl after)
__device__ __forceinline__ void seg_entry2(SegRd& r, int lane, int32_t P, int32_t tl, uint32_t tmask, uint32_t& e1,
                                           uint32_t& e2)
{
    const bool rf = P - r.wlo < 2 * tl;
    r.W = rf ? ((r.W << 32) | r.nx) : r.W;
    r.wlo = rf ? r.wlo - 32 : r.wlo;
    r.nx = sDec.stg[((r.wlo >> 5) - 1) & 15][lane];
    e1 = sDec.tab[(uint32_t)(r.W >> ((P - tl - r.wlo) & 63)) & tmask];
    const int32_t P2 = P - (int32_t)(e1 >> 8);
    e2 = sDec.tab[(uint32_t)(r.W >> ((P2 - tl - r.wlo) & 63)) & tmask];
}
// one table entry (a fixed position refills at most once)
__device__ __forceinline__ uint32_t seg_entry1(SegRd& r, int lane, int32_t P, int32_t tl, uint32_t tmask)
{
    const bool rf = P - r.wlo < tl;
    r.W = rf ? ((r.W << 32) | r.nx) : r.W;
    r.wlo = rf ? r.wlo - 32 : r.wlo;
    r.nx = sDec.stg[((r.wlo >> 5) - 1) & 15][lane];
    return sDec.tab[(uint32_t)(r.W >> ((P - tl - r.wlo) & 63)) & tmask];
}

// 128-bit codeword-start bitmap: bit d = a start at (top - d)
struct SegBm {
    uint64_t q0, q1;
};
__device__ __forceinline__ bool bm_test(const SegBm& b, int32_t d)
{
    const uint64_t w = d < 64 ? b.q0 : b.q1;
    return d >= 0 && d < kSegRec && ((w >> (d & 63)) & 1ull) != 0;
}
// starts recorded above position top - d (bits below d)
__device__ __forceinline__ uint32_t bm_below(const SegBm& b, int32_t d)
{
    const uint64_t m0 = d >= 64 ? ~0ull : (d <= 0 ? 0ull : ((1ull << d) - 1ull));
    const uint64_t m1 = d >= 128 ? ~0ull : (d <= 64 ? 0ull : ((1ull << (d - 64)) - 1ull));
    return (uint32_t)__builtin_popcountll(b.q0 & m0) + (uint32_t)__builtin_popcountll(b.q1 & m1);
}

// Returns false on a malformed section.  tl/minNb: the table in sDec.tab (tl <= kHufLdsLog) and its
// shortest code.  jt01/jt2: the jump table (l1 | l2 << 16, l3).  dst: rs bytes, stream k at k * seg.
// segBuf/segCap: scratch for the segment regions (16-byte aligned).
__device__ __noinline__ bool huf_seg_decode4_wave(unsigned tl, unsigned minNb, const uint8_t* hp, size_t remain,
                                                  uint8_t* dst, uint32_t rs, uint32_t jt01, uint32_t jt2,
                                                  uint8_t* segBuf, size_t segCap, PhaseProf& P, uint32_t diag = 0)
{
    diag = uni(diag);
    const int lane = lane_id();
    tl = uni(tl);
    minNb = uni(minNb);
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    dst = uni(dst);
    rs = uni(rs);
    jt01 = uni(jt01);
    jt2 = uni(jt2);
    segBuf = uni(segBuf);
    segCap = uni((uint64_t)segCap);
    const int k = lane >> 4, j = lane & 15;
    const size_t l1 = jt01 & 0xFFFFu, l2 = jt01 >> 16, l3 = jt2;
    if (l1 + l2 + l3 + 6 > remain) return false;
    const size_t l4 = remain - 6 - l1 - l2 - l3;
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs) return false;
    if (minNb < 1) minNb = 1;
    const size_t so = (k == 0) ? 0 : (k == 1 ? l1 : (k == 2 ? l1 + l2 : l1 + l2 + l3));
    const int32_t sl = (int32_t)((k == 0) ? l1 : (k == 1 ? l2 : (k == 2 ? l3 : l4)));
    const uint32_t nsym = (k == 3) ? rs - 3 * seg : seg;
    const uint8_t* src = hp + 6 + so;
    const uint8_t lastB = sl > 0 ? gb(src + sl - 1) : 0;
    if (ballot(lastB == 0)) return false;
    const int32_t tli = (int32_t)tl;
    const uint32_t tmask = (1u << tl) - 1u;
    const int32_t T = (sl - 1) * 8 + (int32_t)z1::highbit32(lastB);  // stream-relative true start
    // segments: as many as the longest stream allows (>= kSegMinBits each); a region holds the most
    // symbols its segment plus a walk can produce.  The regions together hold about (all bits) /
    // minNb bytes whatever S is: when the scratch is too small, one lane per stream decodes straight
    // into the destination.
    const int32_t Tmax = (int32_t)wave_max((uint32_t)T);
    int S = Tmax / kSegMinBits;
    S = S < 1 ? 1 : (S > kSegMax ? kSegMax : S);
    const int32_t Lmax = (Tmax + S - 1) / S;
    uint32_t R = (uint32_t)((Lmax + kSegRec + 2 * tli) / (int32_t)minNb + 32);
    R = (R + 15u) & ~15u;
    if ((size_t)R * 64u > segCap) S = 1;
    P.count(0);
    SegRd rd;
    const uintptr_t sa = (uintptr_t)src;
    rd.base = (const uint8_t*)(sa & ~(uintptr_t)15);
    rd.off = (int32_t)(sa & 15u);
    rd.end = rd.off + sl;
    rd.W = 0;
    rd.wlo = 0;
    rd.nx = 0;
    rd.wb = 0;
    const int32_t b8 = 8 * rd.off;
    const int32_t L = (T + S - 1) / S;
    const bool active = j < S && T - j * L > 0;        // a segment with bits of its own
    const int32_t hi = active ? b8 + T - j * L : b8;   // segment top (base-relative)
    int32_t lo = active ? b8 + T - (j + 1) * L : b8;  // segment bottom
    lo = lo < b8 ? b8 : lo;
    const bool hasNext = active && j + 1 < S && lo > b8;  // lane j+1 holds the segment below mine
    // region: S == 1 decodes straight into the destination (at most nsym symbols)
    uint8_t* reg = (S == 1) ? dst + (size_t)seg * (size_t)k : segBuf + (size_t)(16 * k + j) * R;
    const uint32_t cap = (S == 1) ? nsym : R;
    // lane state
    bool spec = active && j > 0;   // speculative start: overlap, then record
    bool tstart = !spec;           // output starts at a true position (lane 0, restarted lanes) ...
    int32_t spos = hi;             // ... namely here
    int32_t Pp = spec ? (hi + kSegOv < b8 + T ? hi + kSegOv : b8 + T) : hi;
    bool main = active;            // decoding its segment
    bool done = !active;           // segment decoded and its exit synced
    uint32_t cnt = 0, skip = 0;
    SegBm bm{0, 0};
    // window room a single / a four / an eight-symbol step needs (the reader's refill word stays staged)
    const int32_t G1 = tli + 96, G4 = 4 * tli + 96, G8 = 8 * tli + 96;
    uint4 pf[2];             // the next round's new half window: words [wb - 8, wb)
    bool pe0 = false, pe1 = false;  // ... a piece of it across the stream's first byte
    bool fresh = main;       // the window is staged whole before the first round (and after a restart)
    bool attach = main;      // the reader takes W/nx from the window once staged
    if (main) rd.wb = seg_first_wb(Pp);
    int epochs = 0;
    while (ballot(!done)) {
        if (++epochs > kSegMaxEpochs) return false;
        // ---- main rounds: every live lane decodes its window down to its bottom margin
        while (ballot(main)) {
            P.count(1);
            if (main) {
                if (fresh) {
                    seg_stage_full(rd, rd.wb, lane);
                    fresh = false;
                } else {  // move the window down by half: the prefetched words replace the consumed top
                    rd.wb -= kSegStride;
                    if (pe0) pf[0] = seg_load4(rd, rd.wb);
                    if (pe1) pf[1] = seg_load4(rd, rd.wb + 4);
                    seg_put4(rd.wb, pf[0], lane);
                    seg_put4(rd.wb + 4, pf[1], lane);
                }
                pf[0] = seg_prefetch4(rd, rd.wb - 8, pe0);
                pf[1] = seg_prefetch4(rd, rd.wb - 4, pe1);
            }
            lds_sync();
            if (attach) {
                seg_attach(rd, Pp, lane);
                attach = false;
            }
            P.mark(11);
            const int32_t w32 = 32 * rd.wb;
            // singles: the overlap (no output), the recorded head, the alignment to four, the end
            while (true) {
                const bool ov = main && spec && Pp > hi && Pp - w32 >= G1;
                const bool hd = main && Pp <= hi && Pp > lo && Pp - w32 >= G1 &&
                                ((spec && hi - Pp < kSegRec) || (cnt & 3u) != 0 || Pp - lo < 4 * tli || cnt + 4u > cap);
                const bool act = ov || hd;
                if (!ballot(act)) break;
                P.count(2);
                const uint32_t e = seg_entry1(rd, lane, act ? Pp : rd.wlo + 63, tli, tmask);
                if (act) {
                    if (hd && spec && hi - Pp < kSegRec) {
                        const int32_t d = hi - Pp;
                        const uint64_t bit = 1ull << (d & 63);
                        if (d < 64) bm.q0 |= bit;
                        else bm.q1 |= bit;
                    }
                    if (hd) {
                        if (cnt < cap) gst<uint8_t>(reg + cnt, (uint8_t)e);
                        cnt++;
                    }
                    Pp -= (int32_t)(e >> 8);
                }
            }
            P.mark(12);
            // bodies: eight symbols (two dword stores), then four, while the window and the segment
            // have room for that many codewords of the longest length
            const bool body = main && Pp <= hi && (cnt & 3u) == 0 && !(spec && hi - Pp < kSegRec);
            const int32_t lim8 = body ? max(lo + 8 * tli, w32 + G8) : 0x7FFFFFFF;
            while (true) {
                const bool act = Pp >= lim8 && cnt + 8u <= cap;
                if (!ballot(act)) break;
                P.count(3);
                if (act) {
                    uint32_t e[8];
                    int32_t q = Pp;
#pragma unroll
                    for (int u = 0; u < 8; u += 2) {
                        seg_entry2(rd, lane, q, tli, tmask, e[u], e[u + 1]);
                        q -= (int32_t)(e[u] >> 8) + (int32_t)(e[u + 1] >> 8);
                    }
                    const uint32_t w0 = (e[0] & 0xFFu) | ((e[1] & 0xFFu) << 8) | ((e[2] & 0xFFu) << 16) | (e[3] << 24);
                    const uint32_t w1 = (e[4] & 0xFFu) | ((e[5] & 0xFFu) << 8) | ((e[6] & 0xFFu) << 16) | (e[7] << 24);
                    if (!(diag & 1u)) gst<uint64_t>(reg + cnt, (uint64_t)w0 | ((uint64_t)w1 << 32));
                    cnt += 8;
                    Pp = q;
                }
            }
            const int32_t lim4 = body ? max(lo + 4 * tli, w32 + G4) : 0x7FFFFFFF;
            while (true) {
                const bool act = Pp >= lim4 && cnt + 4u <= cap;
                if (!ballot(act)) break;
                P.count(7);
                if (act) {
                    uint32_t e1, e2, e3, e4;
                    seg_entry2(rd, lane, Pp, tli, tmask, e1, e2);
                    int32_t q = Pp - (int32_t)(e1 >> 8) - (int32_t)(e2 >> 8);
                    seg_entry2(rd, lane, q, tli, tmask, e3, e4);
                    q -= (int32_t)(e3 >> 8) + (int32_t)(e4 >> 8);
                    gst<uint32_t>(reg + cnt, (e1 & 0xFFu) | ((e2 & 0xFFu) << 8) | ((e3 & 0xFFu) << 16) | (e4 << 24));
                    cnt += 4;
                    Pp = q;
                }
            }
            P.mark(13);
            // the last bits of the segment (reached in this round's bodies)
            while (true) {
                const bool act = main && Pp <= hi && Pp > lo && Pp - w32 >= G1 && (Pp - lo < 4 * tli || cnt + 4u > cap);
                if (!ballot(act)) break;
                P.count(4);
                const uint32_t e = seg_entry1(rd, lane, act ? Pp : rd.wlo + 63, tli, tmask);
                if (act) {
                    if (cnt < cap) gst<uint8_t>(reg + cnt, (uint8_t)e);
                    cnt++;
                    Pp -= (int32_t)(e >> 8);
                }
            }
            if (main && Pp <= lo) main = false;
            P.mark(14);
        }
        // ---- sync of the lanes that finished their segment in this epoch: the exit against lane
        // j+1's start (its true start, or its recorded starts: DPP row_shl:1 within the row of 16)
        const SegBm nbm{(uint64_t)dpp<0x101>((uint32_t)bm.q0) | ((uint64_t)dpp<0x101>((uint32_t)(bm.q0 >> 32)) << 32),
                        (uint64_t)dpp<0x101>((uint32_t)bm.q1) | ((uint64_t)dpp<0x101>((uint32_t)(bm.q1 >> 32)) << 32)};
        const bool nTrue = dpp<0x101>(tstart ? 1u : 0u) != 0u;
        const int32_t nPos = (int32_t)dpp<0x101>((uint32_t)spos);
        const bool syncing = !done;
        auto meets = [&](int32_t x) { return nTrue ? x == nPos : bm_test(nbm, lo - x); };
        bool synced = syncing && (!hasNext || meets(Pp));
        bool bad = false, restartNext = false;
        bool walk = syncing && !synced;
        while (ballot(walk)) {  // rare: a fresh window at the walking lane's position each round
            P.count(5);
            if (walk) {
                rd.wb = seg_first_wb(Pp);
                seg_stage_full(rd, rd.wb, lane);
            }
            lds_sync();
            if (walk) seg_attach(rd, Pp, lane);
            const int32_t w32 = 32 * rd.wb;
            while (true) {
                const bool act = walk && Pp - w32 >= G1;
                if (!ballot(act)) break;
                if (act) {
                    if (nTrue ? Pp < nPos : (Pp <= b8 || lo - Pp >= kSegRec)) {
                        walk = false;
                        if (nTrue) bad = true;                  // passed lane j+1's true start: corrupt
                        else if (Pp > b8) restartNext = true;   // lane j+1 decodes again from here
                        else synced = true;                     // the stream ended inside the walk
                    } else {
                        const uint32_t e = seg_entry1(rd, lane, Pp, tli, tmask);
                        if (cnt < cap) gst<uint8_t>(reg + cnt, (uint8_t)e);
                        cnt++;
                        Pp -= (int32_t)(e >> 8);
                        if (meets(Pp)) {
                            synced = true;
                            walk = false;
                        }
                    }
                }
            }
        }
        if (ballot(bad)) return false;
        P.mark(9);
        // deliveries to lane j+1 (DPP row_shr:1): the symbols it drops, or where to decode again from
        const bool endInWalk = synced && hasNext && !nTrue && Pp <= b8;  // lanes below hold nothing
        const uint32_t drop = (synced && hasNext && !nTrue && !endInWalk) ? bm_below(nbm, lo - Pp) : 0u;
        const uint32_t msg = syncing ? ((restartNext || endInWalk) ? 2u : (synced && hasNext ? 1u : 0u)) : 0u;
        const uint32_t inMsg = dpp<0x111>(msg), inDrop = dpp<0x111>(drop), inPos = dpp<0x111>((uint32_t)Pp);
        if (syncing) done = true;
        if (j > 0 && active && inMsg == 1u) skip = inDrop;
        if (j > 0 && active && inMsg == 2u) {  // decode my segment again from the true position
            cnt = 0;
            skip = 0;
            spec = false;
            tstart = true;
            Pp = (int32_t)inPos;
            spos = Pp;
            main = Pp > lo;
            done = false;
            if (main) {
                rd.wb = seg_first_wb(Pp);
                fresh = true;
                attach = true;
            }
        }
    }
    P.mark(15);
    // ---- results: the last segment ends exactly at the stream start; the valid counts add up
    bool bad = false;
    if (active && !hasNext && Pp != b8) bad = true;
    if (active && (skip > cnt || cnt > cap)) bad = true;
    const uint32_t v = (active && !bad) ? cnt - skip : 0u;
    uint32_t incl = v;
    incl += dpp<0x111>(incl);
    incl += dpp<0x112>(incl);
    incl += dpp<0x114>(incl);
    incl += dpp<0x118>(incl);
    const uint32_t tot = (uint32_t)__shfl((int)incl, lane | 15, 64);
    if (ballot(bad || tot != nsym) && !(diag & 4u)) return false;
    if (S == 1 || (diag & 2u)) return true;
    // ---- compaction: every lane copies its valid bytes to the stream's place in the destination
    if (v > 0) {
        const uint8_t* a = reg + skip;
        uint8_t* b = dst + (size_t)seg * (size_t)k + (incl - v);
        uint32_t i = 0;
        for (; i + 64 <= v; i += 64) {
            const uint4 x0 = gld<uint4>(a + i), x1 = gld<uint4>(a + i + 16), x2 = gld<uint4>(a + i + 32),
                        x3 = gld<uint4>(a + i + 48);
            gst<uint4>(b + i, x0);
            gst<uint4>(b + i + 16, x1);
            gst<uint4>(b + i + 32, x2);
            gst<uint4>(b + i + 48, x3);
        }
        for (; i + 16 <= v; i += 16) gst<uint4>(b + i, gld<uint4>(a + i));
        for (; i < v; i++) gst<uint8_t>(b + i, gb(a + i));
    }
    P.mark(10);
    return true;
}

}  // namespace pgn
