// pgn_hufjob.h -- deferred four-stream Huffman sections (large decode batches).
//
// The frame decoder (zstd_decompress_wave in dec_zstd_kernel) decodes every zstd frame of a pass
// except the four Huffman streams of a literals-only last block (HUF_decompress4X1 at the call
// C5.hpp:588-667 makes; on the C5 data these are the M frame and most keys frames, 88 % of a chunk's
// literals): those it leaves as a job -- the streams' places, the destination and a compact copy of
// the decode table -- and dec_huf_kernel decodes them afterwards, one LANE per stream, 16 frames per
// wave, every symbol once from its stream's true start.  The frame decoder's own four-stream path
// (pgn_huf4.h) splits one stream over 16 lanes and decodes every symbol twice (a speculative pass, a
// synchronisation, an exact pass); the lane-per-stream decoder has no speculation and no sync, but
// one lane's stream is ~16k symbols long, so it only pays with thousands of frames in flight
// (launch_decode_impl uses it for large passes).
//
// Compact table (LDS budget: 16 frames x 704 B per wave).  zstd's single-symbol table (HUF_readDTableX1)
// has 2^tl entries; longer codes are canonical and occupy the low indices (weight 1 first), a code of
// length L repeats over 2^(tl-L) entries.  The job keeps three segments of the table at three
// resolutions (pgn_zdec.h job_segments): the entry of a peek p (the stream's next tl bits) is
//     idx = min(p, (p >> d1) + C1, (p >> d2) + C2)
// (round 4 kept two segments, min(p, (p >> d) + Cc): 400-480 entries on the bench's keys / M frames,
// now 190-345).  A table of more than kJobTabUse = 352 entries is decoded in place by the frame decoder.
#pragma once
// included by pgn_zdec.h (after the Huffman table builder; sDec, kHufLdsLog)

namespace pgn {

// kJobTab / kJobTabUse: pgn_zdec.h (the table builder writes a job's compact table for dec_frame_fast)

struct HufJob {
    uint64_t hp;      // the section's jump table; stream k starts at hp + 6 + len[0] + .. + len[k-1]
    uint64_t dst;     // rs literals (stream k: seg = (rs + 3) / 4 of them at dst + k seg; the last rs - 3 seg)
    uint32_t len[4];  // stream bytes
    uint32_t rs;
    uint32_t tl, dd, C1;  // table log; d1 | d2 << 8; C1 (the compact table's segments)
    uint32_t flag;        // 1: pending for dec_huf_kernel (written for every unit of a pass)
    uint32_t C2;
    uint32_t pad[2];
};
static_assert(sizeof(HufJob) == 64, "HufJob header");
constexpr size_t kJobBytes = sizeof(HufJob) + 2 * kJobTab;

// Frame decoder side (wave-uniform): the section at hp (4 streams, jump table jt01 / jt2, table in
// sDec.tab with log tl) becomes job `job`.  Returns false -- and leaves the section to the caller's
// in-place decoder, which then reports any corruption -- when the jump table is inconsistent or the
// compact table exceeds kJobTabUse entries.
__device__ __forceinline__ bool huf_defer_body(uint8_t* job, unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst,
                                              uint32_t rs, uint32_t jt01, uint32_t jt2)
{
    const uint32_t lane = (uint32_t)lane_id();
    job = uni(job);
    tl = uni(tl);
    hp = uni(hp);
    remain = uni((uint64_t)remain);
    dst = uni(dst);
    rs = uni(rs);
    jt01 = uni(jt01);
    jt2 = uni(jt2);
    const uint32_t l1 = jt01 & 0xFFFFu, l2 = jt01 >> 16, l3 = jt2;
    if ((size_t)l1 + l2 + l3 + 6 > remain) return false;
    const uint32_t l4 = (uint32_t)(remain - 6 - l1 - l2 - l3);
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs || tl < 1 || tl > kHufLdsLog) return false;
    // T[d] for d = 0 .. 7: table entries whose code is longer than tl - d bits
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t tsz = 1u << tl;
    for (uint32_t u = lane; u < tsz; u += 64) {
        const uint32_t nb = sDec.tab[u] >> 8;
#pragma unroll
        for (uint32_t d = 1; d < 8; d++) cnt[d] += nb + d > tl;
    }
    uint32_t Td[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Td[d] = wave_sum(cnt[d]);
    const JobSeg sg = job_segments(Td, tl);
    if (sg.size > kJobTabUse) return false;
    uint16_t* tab = (uint16_t*)(job + sizeof(HufJob));
    for (uint32_t j = lane; j < sg.size; j += 64) {
        const uint32_t e = sDec.tab[job_entry_index(sg, j)];
        gst<uint16_t>(tab + j, (uint16_t)((e >> 8) | ((e & 0xFFu) << 8)));
    }
    HufJob* J = (HufJob*)job;
    if (lane == 0) {
        gst<uint64_t>(&J->hp, (uint64_t)hp);
        gst<uint64_t>(&J->dst, (uint64_t)dst);
        gst<uint4>(&J->len[0], make_uint4(l1, l2, l3, l4));
        gst<uint4>(&J->rs, make_uint4(rs, tl, sg.d1 | (sg.d2 << 8), sg.C1));
        gst<uint32_t>(&J->C2, sg.C2);
        gst<uint32_t>(&J->flag, 1u);
    }
    return true;
}
// The job header alone (dec_frame_fast writes the compact table itself, from the table build's ranks):
// the same checks and fields as huf_defer_body, the segments given (kc: d1 | d2 << 8, C1, C2).
__device__ __forceinline__ bool huf_defer_header(uint8_t* job, unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst,
                                                 uint32_t rs, uint32_t jt01, uint32_t jt2, const uint32_t (&kc)[3])
{
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t l1 = jt01 & 0xFFFFu, l2 = jt01 >> 16, l3 = jt2;
    if ((size_t)l1 + l2 + l3 + 6 > remain) return false;
    const uint32_t l4 = (uint32_t)(remain - 6 - l1 - l2 - l3);
    const uint32_t seg = (rs + 3) / 4;
    if (seg * 3 > rs || tl < 1 || tl > kHufLdsLog) return false;
    HufJob* J = (HufJob*)job;
    if (lane == 0) {
        gst<uint64_t>(&J->hp, (uint64_t)hp);
        gst<uint64_t>(&J->dst, (uint64_t)dst);
        gst<uint4>(&J->len[0], make_uint4(l1, l2, l3, l4));
        gst<uint4>(&J->rs, make_uint4(rs, tl, kc[0], kc[1]));
        gst<uint32_t>(&J->C2, kc[2]);
        gst<uint32_t>(&J->flag, 1u);
    }
    return true;
}
__device__ __noinline__ bool huf_defer_section(uint8_t* job, unsigned tl, const uint8_t* hp, size_t remain, uint8_t* dst,
                                               uint32_t rs, uint32_t jt01, uint32_t jt2)
{
    return huf_defer_body(job, tl, hp, remain, dst, rs, jt01, jt2);
}

}  // namespace pgn
