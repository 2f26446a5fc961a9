// pgn_huf4.h -- the four Huffman streams of a zstd literals section (HUF_decompress4X1, the literal
// stage of every ZSTD_decompress call at C5.hpp:588-667 and signal_compression.cpp:112-118),
// decoded by one wave.  Included by pgn_zdec.h after the decoder's LDS (sDec) is declared.
//
// 16 lanes per stream, in rounds.  In a round the 16 lanes of a stream take 16 consecutive windows
// of kWinBits bits below the stream's true position T (lane j: (T - (j+1)W, T - jW]).
//   pass A: every lane decodes its window speculatively from the window top, counting symbols and
//           recording its codeword boundaries in the first kBmpBits bits (a 128-bit bitmap held
//           in the lane's registers);
//   sync:   the true path enters window j at lane j-1's exit; lane j walks from there until it meets
//           one of its recorded boundaries (from there its speculative symbols are the true ones),
//           or decodes the rest of its window itself.  A lane whose exit changed makes its successor
//           walk again; this converges at once in practice (Huffman codes resynchronise within a
//           few codewords) and within 15 iterations always;
//   pass B: every lane decodes again from its true entry, now knowing its output offset (a DPP
//           prefix sum of the symbol counts), and stores its symbols straight to the destination.
// Nothing but the destination is written to HBM.
#pragma once

namespace pgn {

#ifdef PGN_DEBUG_HUF
// diagnostic record buffer: 8 words per record (tag, 7 values), filled by every lane that calls
__device__ uint32_t gHufDbg[1 << 18];
__device__ uint32_t gHufDbgN;
__device__ __forceinline__ void hdbg(uint32_t tag, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                                     uint32_t f, uint32_t g)
{
    const uint32_t i = atomicAdd(&gHufDbgN, 8u);
    if (i + 8 <= (1u << 18)) {
        gHufDbg[i] = tag; gHufDbg[i + 1] = a; gHufDbg[i + 2] = b; gHufDbg[i + 3] = c;
        gHufDbg[i + 4] = d; gHufDbg[i + 5] = e; gHufDbg[i + 6] = f; gHufDbg[i + 7] = g;
    }
}
#endif

// Reader over the lane's staged words: Wd = staged bits [wlo, wlo + 64), nxw = the word below it.
struct StgBits {
    uint64_t Wd;
    int32_t wlo;
    uint32_t nxw;
};
__device__ __forceinline__ void stg_init(StgBits& r, int lane, int32_t x)  // x = q - b8 - tl
{
    int32_t wi = x >> 5;
    wi = wi < 0 ? 0 : (wi > kStgWords - 2 ? kStgWords - 2 : wi);
    r.wlo = 32 * wi;
    r.Wd = (uint64_t)sDec.stg[wi][lane] | ((uint64_t)sDec.stg[wi + 1][lane] << 32);
    r.nxw = sDec.stg[wi > 0 ? wi - 1 : 0][lane];
}
// decode-table entry of the tl bits at local position x (one refill at most: tl <= 11 < 32)
__device__ __forceinline__ uint32_t stg_entry(StgBits& r, int lane, int32_t x, uint32_t tmask)
{
    const bool rf = x < r.wlo;
    r.Wd = rf ? ((r.Wd << 32) | r.nxw) : r.Wd;
    r.wlo = rf ? r.wlo - 32 : r.wlo;
    r.nxw = sDec.stg[r.wlo >= 64 ? (r.wlo >> 5) - 1 : 0][lane];
    return sDec.tab[(uint32_t)(r.Wd >> ((x - r.wlo) & 63)) & tmask];
}

// Two decode-table entries: the codeword at x and the one below it.  One refill check and one
// staged-word prefetch serve both lookups: refilling whenever fewer than tl bits remain above the
// window base keeps both peeks inside the 64-bit window (x - wlo < 32 + tl after a refill, so
// x + tl <= wlo + 54).  Halves the per-symbol refill/prefetch cost of the unpredicated loops.
__device__ __forceinline__ void stg_entry2(StgBits& r, int lane, int32_t x, uint32_t tmask, int32_t tl, uint32_t& e1,
                                           uint32_t& e2)
{
    const bool rf = x - r.wlo < tl;
    r.Wd = rf ? ((r.Wd << 32) | r.nxw) : r.Wd;
    r.wlo = rf ? r.wlo - 32 : r.wlo;
    r.nxw = sDec.stg[r.wlo >= 64 ? (r.wlo >> 5) - 1 : 0][lane];
    e1 = sDec.tab[(uint32_t)(r.Wd >> ((x - r.wlo) & 63)) & tmask];
    const int32_t x2 = x - (int32_t)(e1 >> 8);
    e2 = sDec.tab[(uint32_t)(r.Wd >> ((x2 - r.wlo) & 63)) & tmask];
}

// Returns false on a malformed section.  jt = the jump table's three stream sizes (l1 | l2 << 16,
// l3), read by the caller (remain >= 6).
__device__ __noinline__ bool huf_decode4_wave(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                              uint32_t jt01, uint32_t jt2, PhaseProf& P)
{
    const int lane = lane_id();
    tl = uni(tl);
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    dst = uni(dst);
    rs = uni(rs);
    jt01 = uni(jt01);
    jt2 = uni(jt2);
    const int k = lane >> 4, j = lane & 15;
    const size_t l1 = jt01 & 0xFFFFu, l2 = jt01 >> 16, l3 = jt2;
    if (l1 + l2 + l3 + 6 > remain) return false;
    const size_t l4 = remain - 6 - l1 - l2 - l3;
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs) return false;
    const size_t so = (k == 0) ? 0 : (k == 1 ? l1 : (k == 2 ? l1 + l2 : l1 + l2 + l3));
    const int32_t sl = (int32_t)((k == 0) ? l1 : (k == 1 ? l2 : (k == 2 ? l3 : l4)));
    const uint32_t nsym = (k == 3) ? rs - 3 * seg : seg;
    const uint8_t* src = hp + 6 + so;
    const uint8_t lastB = sl > 0 ? gb(src + sl - 1) : 0;
    if (ballot(lastB == 0)) return false;
    uint8_t* sdst = dst + (size_t)seg * (size_t)k;
    const uint32_t tmask = (1u << tl) - 1u;
    const int32_t tli = (int32_t)tl;
    int32_t T = (sl - 1) * 8 + (int32_t)z1::highbit32(lastB);  // the stream's true position
    uint32_t produced = 0;                                     // symbols of the stream stored so far
    // staged bytes of the round: loaded one round ahead from the estimate of the next round's
    // position (T drops by 16W, minus at most tl - 1 bits; round_base leaves room for both)
    int32_t base = round_base(T - j * kWinBits);
    uint4 nx[kStgWords / 4];
    round_load(nx, src, sl, base);
#ifdef PGN_DEBUG_HUF
    hdbg(1, (uint32_t)k, (uint32_t)j, (uint32_t)T, (uint32_t)sl, nsym, tl, rs);
#endif
    while (ballot(T > 0)) {
        P.count(0);
        const int32_t hi = T - j * kWinBits;
        const int32_t lo = (hi - kWinBits > 0) ? hi - kWinBits : 0;
        const int32_t b8 = 8 * base;
#pragma unroll
        for (int i = 0; i < kStgWords / 4; i++) {
            sDec.stg[4 * i][lane] = nx[i].x;
            sDec.stg[4 * i + 1][lane] = nx[i].y;
            sDec.stg[4 * i + 2][lane] = nx[i].z;
            sDec.stg[4 * i + 3][lane] = nx[i].w;
        }
        uint64_t bm0 = 0, bm1 = 0;  // boundary bitmap: bit d = codeword start at hi - d (d < 128)
        const int32_t nextT = T - 16 * kWinBits;
        if (ballot(nextT > 0)) {  // next round's bytes, in flight during this one
            base = round_base(nextT - j * kWinBits);
            round_load(nx, src, sl, base);
        }
        lds_sync();
        // ---- pass A: speculative decode of (lo, hi]: symbol count c, exit q
        // lanes 1..15 start kOvBits above their window (inside the staged bytes: 8 * base + 32 *
        // kStgWords >= hi + 65), so the speculative path has usually merged with the true one by hi
        // and the sync below finds the true entry among the recorded boundaries without a walk
        int32_t q = (j == 0 || hi <= lo) ? hi : hi + kOvBits;
        uint32_t c = 0;
        {
            StgBits r;
            stg_init(r, lane, q - b8 - tli);
            while (ballot(q > hi)) {  // overlap: decoded, neither counted nor recorded
                P.count(1);
                uint32_t e[2];
                stg_entry2(r, lane, q - b8 - tli, tmask, tli, e[0], e[1]);
#pragma unroll
                for (int u = 0; u < 2; u++) q = q > hi ? q - (int32_t)(e[u] >> 8) : q;
            }
            while (ballot(q > lo && hi - q < kBmpBits)) {
                P.count(2);
                uint32_t e[2];
                stg_entry2(r, lane, q - b8 - tli, tmask, tli, e[0], e[1]);
#pragma unroll
                for (int u = 0; u < 2; u++) {  // the second entry is only used if the first was
                    const bool act = q > lo && hi - q < kBmpBits;
                    const int32_t d = hi - q;
                    const uint64_t bit = 1ull << (d & 63);
                    bm0 |= (act && d < 64) ? bit : 0ull;
                    bm1 |= (act && d >= 64) ? bit : 0ull;
                    q = act ? q - (int32_t)(e[u] >> 8) : q;
                    c += act ? 1u : 0u;
                }
            }
            // every active lane has >= 4 * tl bits left: four symbols without a bound check
            while (ballot(q > lo) && !ballot(q > lo && q - lo < 4 * tli)) {
                P.count(3);
                const bool act = q > lo;
                int32_t qq = q;
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    uint32_t e1, e2;
                    stg_entry2(r, lane, qq - b8 - tli, tmask, tli, e1, e2);
                    qq -= (int32_t)(e1 >> 8) + (int32_t)(e2 >> 8);
                }
                q = act ? qq : q;
                c += act ? 4u : 0u;
            }
            while (ballot(q > lo)) {
                P.count(4);
#pragma unroll
                for (int v = 0; v < 2; v++) {
                    uint32_t e[2];
                    stg_entry2(r, lane, q - b8 - tli, tmask, tli, e[0], e[1]);
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const bool act = q > lo;
                        q = act ? q - (int32_t)(e[u] >> 8) : q;
                        c += act ? 1u : 0u;
                    }
                }
            }
        }
        P.mark(11);
        // ---- sync: true entries, symbol counts and exits
        // (DPP reads a disabled source lane as 0: the moves run on the full wave, outside any branch)
        const int32_t prevQ = (int32_t)dpp<kDppRowShr1>((uint32_t)q);
        int32_t entry = (j == 0) ? hi : prevQ;
        uint32_t cnt = c;  // lane 0 starts on the true path
        int32_t ex = q;
        bool need = j > 0;
        for (int it = 0; it < 16; it++) {
            P.count(5);
            if (need) {
                int32_t p = entry;
                uint32_t w = 0;
                // a recorded boundary at p (none lies at or below lo: kBmpBits < kWinBits)
                auto recorded = [&](int32_t pp) {
                    const int32_t d = hi - pp;
                    return d < kBmpBits && (((d < 64 ? (bm0 >> d) : (bm1 >> (d - 64))) & 1ull) != 0);
                };
                bool synced = recorded(p);
                if (!synced && p > lo) {  // walk the true path until it meets a recorded boundary
                    StgBits r;
                    stg_init(r, lane, p - b8 - tli);
                    do {
                        const uint32_t e = stg_entry(r, lane, p - b8 - tli, tmask);
                        p -= (int32_t)(e >> 8);
                        w++;
                    } while (p > lo && !(synced = recorded(p)));
                }
                if (synced) {
                    const int32_t d = hi - p;
                    // boundaries recorded below d (d < 128 here)
                    const uint64_t m0 = d >= 64 ? ~0ull : ((1ull << d) - 1ull);
                    const uint64_t m1 = d <= 64 ? 0ull : ((1ull << (d - 64)) - 1ull);
                    const uint32_t idx = (uint32_t)__builtin_popcountll(bm0 & m0) + (uint32_t)__builtin_popcountll(bm1 & m1);
                    cnt = w + c - idx;
                    ex = q;
                } else {
                    cnt = w;
                    ex = p;
                }
            }
#ifdef PGN_PROFILE
            P.count(6, wave_max(need ? cnt : 0u) > 0 ? 1u : 0u);  // sync iterations with any walking lane
#endif
            const int32_t prevEx = (int32_t)dpp<kDppRowShr1>((uint32_t)ex);
            const int32_t ne = (j == 0) ? hi : prevEx;
            need = (j > 0) && (ne != entry);
            entry = ne;
            if (!ballot(need)) break;
        }
        P.mark(12);
        // ---- output offsets: DPP prefix over the stream's 16 lanes (one row)
        uint32_t incl = cnt;
        incl += dpp<kDppRowShr1>(incl);
        incl += dpp<kDppRowShr2>(incl);
        incl += dpp<kDppRowShr4>(incl);
        incl += dpp<kDppRowShr8>(incl);
        const uint32_t tot = (uint32_t)__shfl((int)incl, lane | 15, 64);
        const int32_t Tn = __shfl(ex, lane | 15, 64);
#ifdef PGN_DEBUG_HUF
        if (produced < 2000) hdbg(2 + 16 * k + 256 * j, (uint32_t)T, (uint32_t)hi, (uint32_t)lo, c, (uint32_t)q,
                                  (uint32_t)entry, cnt | ((uint32_t)ex << 16));
#endif
        if (ballot(produced + tot > nsym)) return false;
        // ---- pass B: decode again from the true entry, storing the symbols
        {
            uint8_t* out = sdst + produced + (incl - cnt);
            int32_t p = entry;
            StgBits r;
            stg_init(r, lane, p - b8 - tli);
            // Lanes that are done keep decoding at their fixed position (their reader stays valid: a
            // fixed position refills at most once) and store nothing; the trip counts are wave-uniform,
            // so the loops have no divergent region and the loop-carried state needs no copies.
            const uint32_t my4 = cnt >> 2, myTail = cnt & 3u;
            const uint32_t n4 = wave_max(my4), nTail = wave_max(myTail);
            for (uint32_t g = 0; g < n4; g++) {
                P.count(7);
                const bool act = g < my4;
                uint32_t word = 0;
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    uint32_t e1, e2;
                    stg_entry2(r, lane, p - b8 - tli, tmask, tli, e1, e2);
                    p -= act ? (int32_t)(e1 >> 8) + (int32_t)(e2 >> 8) : 0;
                    word |= ((e1 & 0xFFu) | ((e2 & 0xFFu) << 8)) << (16 * u);
                }
                if (act) gst<uint32_t>(out + 4u * g, word);
            }
            out += 4u * my4;
            for (uint32_t g = 0; g < nTail; g++) {
                P.count(8);
                const bool act = g < myTail;
                const uint32_t e = stg_entry(r, lane, p - b8 - tli, tmask);
                p -= act ? (int32_t)(e >> 8) : 0;
                if (act) gst<uint8_t>(out + g, (uint8_t)e);
            }
        }
        P.mark(8);
        produced += tot;
        T = Tn;
        lds_sync();
    }
    // every stream must end exactly at its first bit with all its symbols
#ifdef PGN_DEBUG_HUF
    hdbg(3, (uint32_t)k, (uint32_t)j, (uint32_t)T, produced, nsym, 0, 0);
#endif
    return !ballot(T != 0 || produced != nsym);
}

}  // namespace pgn
