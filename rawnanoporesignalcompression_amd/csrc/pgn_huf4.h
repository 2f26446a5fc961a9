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

// Reader over the lane's staged words.  Wd holds the staged bits [32 (row + 1), 32 (row + 1) + 64) of
// the round's window, u is the shift of the next codeword's tl-bit peek inside Wd (the codeword's top
// bit is at local position u + tl + 32 (row + 1)), nxw is staged word `row` (the next refill).  A
// refill check every two codewords keeps both peeks inside Wd (u >= tl after it; u < tl + 32 <= 43
// so u + tl <= 54).  Rows below 0 read the decode table in front of the staging rows: only a path
// that has left the stream's staged bits does that (the rows in front of the staging are LDS of
// the same workgroup), and it never uses the bits.
struct HufRd {
    uint64_t Wd;
    int32_t u;
    int32_t row;
    uint32_t nxw;
};
// Staging rows: row r of lane l at stg[64 r + l] (word-major, so the lanes of a row hit distinct
// banks).  The 16-lanes-per-stream decoder uses sDec.stg; the cooperative one (64 lanes per stream,
// one wave per stream) gives each wave its own rows in its kernel's LDS, passed as an LDS pointer (an
// LDS variable named by non-kernel functions of several kernels would move the others' LDS behind
// a per-kernel offset table).
__device__ __forceinline__ uint32_t stg_word(const lds_u32* stg, int32_t row, int lane)
{
    return stg[64 * row + lane];
}
__device__ __forceinline__ void rd_init(HufRd& r, const lds_u32* stg, int lane, int32_t x)  // x = q - b8 - tl
{
    int32_t wi = x >> 5;
    wi = wi < 0 ? 0 : (wi > kStgWords - 2 ? kStgWords - 2 : wi);
    r.Wd = (uint64_t)stg_word(stg, wi, lane) | ((uint64_t)stg_word(stg, wi + 1, lane) << 32);
    r.u = x - 32 * wi;
    r.row = wi - 1;
    r.nxw = stg_word(stg, r.row, lane);
}
__device__ __forceinline__ void rd_refill(HufRd& r, const lds_u32* stg, int lane, int32_t tl)
{
    const bool rf = r.u < tl;
    r.Wd = rf ? ((r.Wd << 32) | r.nxw) : r.Wd;
    r.u += rf ? 32 : 0;
    r.row -= rf ? 1 : 0;
    r.nxw = stg_word(stg, r.row, lane);
}
// decode-table entry (symbol | nbBits << 8) of the next codeword
__device__ __forceinline__ uint32_t rd_entry(const HufRd& r, uint32_t tmask)
{
    return sDec.tab[(uint32_t)(r.Wd >> r.u) & tmask];
}
__device__ __forceinline__ uint32_t rd_nbits(const HufRd& r, uint32_t tmask)
{
    return (uint32_t)(reinterpret_cast<const uint8_t*>(sDec.tab))[2u * ((uint32_t)(r.Wd >> r.u) & tmask) + 1u];
}
// z = u + 32 row: the next codeword's top position is z + (tl + b8 + 32)
__device__ __forceinline__ int32_t rd_z(const HufRd& r) { return r.u + 32 * r.row; }

// the value of lane j - 1 of the same stream (lane 0 of a stream reads a value it does not use)
template <int LPS>
__device__ __forceinline__ int32_t prev_lane(int32_t x)
{
    if (LPS == 16) return (int32_t)dpp<kDppRowShr1>((uint32_t)x);
    return __shfl_up(x, 1, 64);
}

// Recorded codeword starts: the first kRecSyms starts at or below a lane's window top, as distances
// below the top, one byte each (0xFF = none; a distance is at most tl - 1 + 19 * 11 < 255).
constexpr int kRecSyms = 20;
struct RecStarts {
    uint32_t w[kRecSyms / 4];
};
// number of recorded starts before the one at distance d (-1: none recorded at d).  The distances
// increase, so at most one byte matches; a word's lowest zero byte after the XOR is exact.
__device__ __forceinline__ int32_t rec_index(const RecStarts& R, int32_t d)
{
    if (d < 0 || d > 254) return -1;
    const uint32_t rep = (uint32_t)d * 0x01010101u;
#pragma unroll
    for (int i = 0; i < kRecSyms / 4; i++) {
        const uint32_t x = R.w[i] ^ rep;
        const uint32_t z = (x - 0x01010101u) & ~x & 0x80808080u;
        if (z) return 4 * i + (int32_t)(__builtin_ctz(z) >> 3);
    }
    return -1;
}

// Returns false on a malformed section.  jt = the jump table's three stream sizes (l1 | l2 << 16,
// l3), read by the caller (remain >= 6).
//
// LPS = lanes per stream: 16 (one wave decodes the four streams, huf_decode4_wave) or 64 (the
// cooperative decoder: wave kStream decodes stream kStream with all its lanes; coopStg = its rows,
// with two spare rows in front: a refill reads at most two rows below row 0).
constexpr int kCoopWaves = 4;
constexpr int kCoopStgWords = (kStgWords + 2) * 64;  // per wave

template <int LPS>
__device__ __forceinline__ bool huf_decode_lanes(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                                 uint32_t jt01, uint32_t jt2, int kStream, lds_u32* coopStg,
                                                 PhaseProf& P)
{
    static_assert(LPS == 16 || LPS == 64, "16 or 64 lanes per stream");
    const int lane = lane_id();
    lds_u32* stg = LPS == 16 ? (lds_u32*)&sDec.stg[0][0] : coopStg;
    tl = uni(tl);
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    dst = uni(dst);
    rs = uni(rs);
    jt01 = uni(jt01);
    jt2 = uni(jt2);
    const int k = LPS == 16 ? lane >> 4 : kStream, j = LPS == 16 ? lane & 15 : lane;
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
            stg[64 * (4 * i) + lane] = nx[i].x;
            stg[64 * (4 * i + 1) + lane] = nx[i].y;
            stg[64 * (4 * i + 2) + lane] = nx[i].z;
            stg[64 * (4 * i + 3) + lane] = nx[i].w;
        }
        const int32_t nextT = T - LPS * kWinBits;
        if (ballot(nextT > 0)) {  // next round's bytes, in flight during this one
            base = round_base(nextT - j * kWinBits);
            round_load(nx, src, sl, base);
        }
        lds_sync();
        // ---- pass A: speculative decode of (lo, hi]: symbol count c, exit q, the first kRecSyms
        // codeword starts at or below hi (distances hi - q, one byte each; 0xFF = none)
        // lanes 1..15 start kOvBits above their window (inside the staged bytes: 8 * base + 32 *
        // kStgWords >= hi + 65), so the speculative path has usually merged with the true one by hi
        // and the sync below finds the true entry among the recorded starts without a walk.
        // Positions are kept as z = q - K0 (the reader's u + 32 row).
        const int32_t K0 = tli + b8 + 32;
        const int32_t zHi = hi - K0, zLo = lo - K0;
        uint32_t c = 0;
        RecStarts rec;
        int32_t q;
        {
            HufRd r;
            rd_init(r, stg, lane, ((j == 0 || hi <= lo) ? hi : hi + kOvBits) - b8 - tli);
            while (ballot(rd_z(r) > zHi)) {  // overlap: decoded, neither counted nor recorded
                P.count(1);
                rd_refill(r, stg, lane, tli);
#pragma unroll
                for (int v = 0; v < 2; v++) {
                    const uint32_t nb = rd_nbits(r, tmask);
                    r.u -= rd_z(r) > zHi ? (int32_t)nb : 0;
                }
            }
            P.count(2);
#pragma unroll
            for (int i = 0; i < kRecSyms; i++) {  // the first kRecSyms codewords: recorded and counted
                if ((i & 1) == 0) rd_refill(r, stg, lane, tli);
                const int32_t z = rd_z(r);
                const bool act = z > zLo;
                const uint32_t d = act ? (uint32_t)(zHi - z) : 0xFFu;
                rec.w[i >> 2] = (i & 3) ? (rec.w[i >> 2] | (d << (8 * (i & 3)))) : d;
                const uint32_t nb = rd_nbits(r, tmask);
                r.u -= act ? (int32_t)nb : 0;
                c += act ? 1u : 0u;
            }
            // every active lane has >= 4 * tl bits left: four symbols, lanes that are done frozen
            while (ballot(rd_z(r) > zLo) && !ballot(rd_z(r) > zLo && rd_z(r) - zLo < 4 * tli)) {
                P.count(3);
                const bool act = rd_z(r) > zLo;
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    if ((v & 1) == 0) rd_refill(r, stg, lane, tli);
                    const uint32_t nb = rd_nbits(r, tmask);
                    r.u -= act ? (int32_t)nb : 0;
                }
                c += act ? 4u : 0u;
            }
            while (ballot(rd_z(r) > zLo)) {
                P.count(4);
                rd_refill(r, stg, lane, tli);
#pragma unroll
                for (int v = 0; v < 2; v++) {
                    const bool act = rd_z(r) > zLo;
                    const uint32_t nb = rd_nbits(r, tmask);
                    r.u -= act ? (int32_t)nb : 0;
                    c += act ? 1u : 0u;
                }
            }
            q = rd_z(r) + K0;
        }
        P.mark(11);
        // ---- sync: true entries, symbol counts and exits
        // (DPP reads a disabled source lane as 0: the moves run on the full wave, outside any branch)
        const int32_t prevQ = prev_lane<LPS>(q);
        int32_t entry = (j == 0) ? hi : prevQ;
        uint32_t cnt = c;  // lane 0 starts on the true path
        int32_t ex = q;
        // Only lanes whose window is not empty (hi > 0) take part: the stream's last such lane ends at
        // its first bit, and the empty ones above it hold no symbols.  Every iteration settles at
        // least one more lane, so LPS iterations always converge.
        bool need = j > 0 && hi > 0;
        for (int it = 0; it < LPS; it++) {
            P.count(5);
            if (need) {
                int32_t p = entry;
                uint32_t w = 0;
                int32_t idx = rec_index(rec, hi - p);
                if (idx < 0 && p > lo) {  // walk the true path until it meets a recorded start
                    HufRd r;
                    rd_init(r, stg, lane, p - b8 - tli);
                    do {
                        rd_refill(r, stg, lane, tli);
                        const uint32_t nb = rd_nbits(r, tmask);
                        r.u -= (int32_t)nb;
                        p -= (int32_t)nb;
                        w++;
                    } while (p > lo && (idx = rec_index(rec, hi - p)) < 0);
                }
                if (idx >= 0) {
                    cnt = w + c - (uint32_t)idx;
                    ex = q;
                } else {
                    cnt = w;
                    ex = p;
                }
            }
#ifdef PGN_PROFILE
            P.count(6, wave_max(need ? cnt : 0u) > 0 ? 1u : 0u);  // sync iterations with any walking lane
#endif
            const int32_t prevEx = prev_lane<LPS>(ex);
            const int32_t ne = (j == 0) ? hi : prevEx;
            need = (j > 0) && hi > 0 && (ne != entry);
            entry = ne;
            if (!ballot(need)) break;
        }
        P.mark(12);
        // ---- output offsets: DPP prefix over the stream's 16 lanes (one row)
        uint32_t incl = cnt;
        uint32_t tot;
        int32_t Tn;
        const uint64_t live = ballot(hi > 0);  // lanes with a window (contiguous from j = 0 in each stream)
        if (LPS == 16) {
            incl += dpp<kDppRowShr1>(incl);
            incl += dpp<kDppRowShr2>(incl);
            incl += dpp<kDppRowShr4>(incl);
            incl += dpp<kDppRowShr8>(incl);
            tot = (uint32_t)__shfl((int)incl, lane | 15, 64);
            const uint32_t rowLive = (uint32_t)(live >> (16 * k)) & 0xFFFFu;
            const int jl = rowLive ? 31 - __builtin_clz(rowLive) : 0;
            const int32_t exl = __shfl(ex, 16 * k + jl, 64);
            Tn = rowLive ? exl : T;  // a finished stream stays where it ended
        } else {
            incl = wave_incl_sum(incl);
            tot = readlane_u32(incl, 63);
            const int jl = live ? 63 - __builtin_clzll(live) : 0;
            const int32_t exl = (int32_t)__builtin_amdgcn_readlane((int)ex, jl);
            Tn = live ? exl : T;
        }
#ifdef PGN_DEBUG_HUF
        if (produced < 2000) hdbg(2 + 16 * k + 256 * j, (uint32_t)T, (uint32_t)hi, (uint32_t)lo, c, (uint32_t)q,
                                  (uint32_t)entry, cnt | ((uint32_t)ex << 16));
#endif
        if (ballot(produced + tot > nsym)) return false;
        // ---- pass B: decode again from the true entry, storing the symbols
        {
            uint8_t* out = sdst + produced + (incl - cnt);
            HufRd r;
            rd_init(r, stg, lane, entry - b8 - tli);
            // Lanes that are done keep their position (their codeword lengths count as 0) and store
            // nothing; the trip counts are wave-uniform, so the loops have no divergent region.
            const uint32_t my4 = cnt >> 2, myTail = cnt & 3u;
            const uint32_t n4 = wave_max(my4), nTail = wave_max(myTail);
            for (uint32_t g = 0; g < n4; g++) {
                P.count(7);
                const bool act = g < my4;
                const uint32_t w8 = act ? 8u : 0u;  // nbBits field width: 0 keeps a finished lane in place
                uint32_t e[4];
#pragma unroll
                for (int v = 0; v < 4; v++) {
                    if ((v & 1) == 0) rd_refill(r, stg, lane, tli);
                    e[v] = rd_entry(r, tmask);
                    r.u -= (int32_t)__builtin_amdgcn_ubfe(e[v], 8u, w8);
                }
                const uint32_t word = __builtin_amdgcn_perm(e[1], e[0], 0x0C0C0400u) |
                                      (__builtin_amdgcn_perm(e[3], e[2], 0x0C0C0400u) << 16);
                if (act) gst<uint32_t>(out + 4u * g, word);
            }
            out += 4u * my4;
            for (uint32_t g = 0; g < nTail; g++) {
                P.count(8);
                const bool act = g < myTail;
                rd_refill(r, stg, lane, tli);
                const uint32_t e = rd_entry(r, tmask);
                r.u -= act ? (int32_t)(e >> 8) : 0;
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

__device__ __noinline__ bool huf_decode4_wave(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                              uint32_t jt01, uint32_t jt2, PhaseProf& P)
{
    return huf_decode_lanes<16>(tl, hp, remain, dst, rs, jt01, jt2, 0, nullptr, P);
}
// one stream of the section with all 64 lanes (cooperative decoder: wave kStream of the workgroup,
// stg = its staging rows)
__device__ __noinline__ bool huf_decode1of4_wave64(unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst, uint32_t rs,
                                                   uint32_t jt01, uint32_t jt2, int kStream, lds_u32* stg, PhaseProf& P)
{
    return huf_decode_lanes<64>(tl, hp, remain, dst, rs, jt01, jt2, kStream, stg, P);
}

}  // namespace pgn
