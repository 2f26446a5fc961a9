// pgn_kernels.hip -- gfx950 kernels and the C ABI (include/pgnano_hip.h) of the C5 codec.
//
// Layout (DESIGN.md "Data layout in HBM"): one 64-lane workgroup per resident slot; each slot owns a
// fixed scratch window in HBM (its five streams, hash table, literal/sequence staging) and walks the
// chunks blockIdx.x, blockIdx.x + gridDim.x, ...  Chunks are independent (the delta restarts at 0
// and every zstd frame is self-contained, C5.hpp:302-309), so there is no inter-workgroup traffic.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "../../include/pgnano_hip.h"
#include "../../include/pgnano_pod5.h"
#include "pgn_c5.h"
#include "pgn_internal.h"
#include "pgn_vbz.h"
#include "pgn_variants.h"
#include "pgn_zdec.h"
#include "pgn_zenc.h"

namespace pgn {

// Chunks up to kPassSamples take the batched passes, whose per-chunk buffers are spaced for that
// many samples; larger ones (up to PGN_MAX_CHUNK_SAMPLES) take the large-chunk pass, whose slot
// buffers are spaced for the largest chunk of the call (launch_large_*).
constexpr uint32_t kPassSamples = 262144;
static_assert(PGN_MAX_CHUNK_SAMPLES >= kPassSamples, "chunk limits");
// literals and sequences live per zstd block (<= 128 KiB); a frame's blocks reuse them
constexpr uint32_t kMaxEncSeq = (uint32_t)z1::kMaxSrc / 4 + 2;  // every match covers >= 4 bytes
constexpr uint32_t kMaxDecSeq = (uint32_t)z1::kMaxSrc / 3 + 2;  // any valid block: matches >= 3 bytes
// every stream of the largest chunk fits one encoder frame (its svb16 buffer, ~2.13 n, the largest)
static_assert((size_t)PGN_MAX_CHUNK_SAMPLES * 9 / 4 + 64 <= kMaxFrameBytes, "frame index field");
constexpr int kStreams = 5;
// Codecs of a batch call: the pgnano C5 variant (5 zstd frames per chunk) and the pod5 VBZ codec
// (one zstd frame per chunk).  Both share the per-chunk buffers and the zstd kernels.
enum Codec : int { kCodecC5 = 0, kCodecVbz = 1, kCodecC4 = 2, kCodecC1 = 3, kCodecC2 = 4, kCodecC3 = 5, kCodecVbz0 = 6 };

__host__ __device__ constexpr size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Capacity of C5 stream s of a chunk of at most capN samples: keys n/4, S n/2, M/Ll/Lh n.  The
// stream area of a chunk (3.75 capN) also holds its VBZ / C1 svb16 buffer (<= 2.13 n) and the other
// variants' streams.
__host__ __device__ constexpr uint32_t stream_cap(int s, uint32_t capN = kPassSamples)
{
    return s == 0 ? capN / 4 + 1 : (s == 1 ? capN / 2 + 1 : capN);
}
__host__ __device__ constexpr size_t stream_pad(int s, uint32_t capN = kPassSamples)
{
    return align_up((size_t)stream_cap(s, capN) + 64, 256);
}
// byte offset of stream s inside a chunk's stream area
__host__ __device__ constexpr size_t stream_off(int s, uint32_t capN = kPassSamples)
{
    size_t o = 0;
    for (int t = 0; t < s; t++) o += stream_pad(t, capN);
    return o;
}
__host__ __device__ constexpr size_t chunk_stream_bytes(uint32_t capN) { return stream_off(kStreams, capN); }
constexpr size_t kChunkStreamBytes = chunk_stream_bytes(kPassSamples);
// ZSTD_COMPRESSBOUND (the frame of a stream never exceeds it)
__host__ __device__ constexpr size_t frame_bound(size_t n)
{
    return n + (n >> 8) + (n < (128u << 10) ? (((128u << 10) - n) >> 11) : 0);
}
__host__ __device__ constexpr size_t frame_pad(int s) { return align_up(frame_bound(stream_cap(s)) + 64, 256); }
__host__ __device__ constexpr size_t frame_off(int s)
{
    size_t o = 0;
    for (int t = 0; t < s; t++) o += frame_pad(t);
    return o;
}
constexpr size_t kChunkFrameBytes = frame_off(kStreams);

// ---------------------------------------------------------------------------------------------
// Scratch of one resident zstd-encode workgroup ("slot")
// ---------------------------------------------------------------------------------------------
struct EncLayout {
    size_t ht, lit, seqs, codes, seqSection, seqWork, huf, bytes;
};
__host__ __device__ inline EncLayout enc_layout()
{
    EncLayout l{};
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o = align_up(o + n + 64, 256); return r; };
    l.ht = take((size_t)4 << 15);
    l.lit = take(z1::kMaxSrc);
    l.seqs = take(sizeof(z1::Seq) * kMaxEncSeq);
    l.codes = take(3 * (size_t)kMaxEncSeq);
    l.seqSection = take(16 + 10 * (size_t)kMaxEncSeq + 1024);
    l.seqWork = take(sizeof(z1::SeqWork));
    l.huf = take(2 * 256 * 4);
    l.bytes = o;
    return l;
}

struct DecLayout {
    size_t lit, seqs, tables, htab, bytes;
};
__host__ __device__ inline DecLayout dec_layout()
{
    DecLayout l{};
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o = align_up(o + n + 64, 256); return r; };
    l.lit = take(z1::kMaxSrc);
    l.seqs = take(12 * (size_t)kMaxDecSeq);
    l.tables = take(4 * ((size_t)kSeqTab + 4));
    l.htab = take(2u << z1::kHufTableLogMax);
    l.bytes = o;
    return l;
}
// A chunk's intermediate (the decoded frames back to back) holds 2.25 capN + 1,024 bytes: the most
// any blob of a chunk of n <= capN samples holds when its frames decode to what its merge consumes --
// C5 / C4: n/4 key bytes + 2 bytes per sample at most (a class-3 sample), every one of its S / M /
// class-3 bytes standing for one sample; C1 / C2 / C3: n/8 + 2 n; VBZ0 n/4 + 2 n; VBZ's svb16 buffer
// n/8 + 2 n + 16 padding bytes -- plus slack for trailing bytes ("Remaining data").  Frames claiming
// more go through over_claim_status (the reference's own outcome for them, decided without decoding).
__host__ __device__ constexpr size_t inter_cap(uint32_t capN) { return (size_t)capN * 9 / 4 + 1024; }
// svb16::decode_input_buffer_padding_byte_count() on x86-64 (svb16/decode.hpp:16-23): the VBZ
// intermediate is the frame content plus 16 bytes, and ZSTD_decompress may fill them.
constexpr size_t kVbzPadding = 16;
constexpr uint64_t kAllocLimit = (uint64_t)1 << 40;  // a decode intermediate above this is an allocation failure (PGN_ERR_ALLOC)
__host__ __device__ constexpr size_t chunk_inter_bytes(uint32_t capN) { return align_up(inter_cap(capN) + 64, 256); }
// per-chunk decode buffers of the passes in flight (intermediates, records, Huffman jobs), all
// buffers together
constexpr size_t kDecBufferBudget = (size_t)32 << 30;
constexpr int kMaxDecBufs = 4;  // decode pass buffers in rotation (pgn_ctx::decBufs)

// Work-unit order of the per-stream kernels: the large streams first (M, S, keys, Llow, Lhigh), so
// the dynamic queue ends with short units.
__device__ __forceinline__ int unit_stream(uint32_t k) { return (int)((0x43012u >> (4 * k)) & 0xFu); }

// ---------------------------------------------------------------------------------------------
// Encode: split -> per-stream zstd -> assemble, over a sub-batch of G chunks (chunk g = base + g)
// ---------------------------------------------------------------------------------------------
struct EncArgs {
    size_t nchunks;
    const int16_t* samples;
    const uint64_t* sampleOffsets;
    const uint32_t* sampleCounts;
    uint8_t* out;
    const uint64_t* outOffsets;
    const uint64_t* outCaps;
    uint64_t* outSizes;
    int32_t* status;
    uint64_t* stats;
    uint8_t* streams;    // G * kChunkStreamBytes
    uint8_t* frames;     // G * kChunkFrameBytes
    uint32_t* sizes;     // [G][5] raw stream sizes; sizes[g*5] = ~0u marks an unsupported chunk
    uint32_t* fsizes;    // [G][5] frame sizes
    uint8_t* slotScratch;
    size_t slotBytes;
    uint32_t* epochs;
    uint32_t* queue;     // work counter of this sub-batch
    uint64_t* prof;
    size_t base, G;
    uint32_t nu;         // zstd work units per chunk: 5 (C5) or 1 (VBZ)
    // fused kernels: slot buffers spaced for capN samples; chunk u of the queue is list[u] (the
    // large-chunk pass) or u
    uint32_t capN;
    const uint32_t* list;
    uint64_t* lookback;  // small batches: the range split's published words (kSplitRanges x 2 per chunk)
    uint64_t epoch;      // this call's tag in those words (bits 48..63)
};

__global__ __launch_bounds__(64) void enc_split_kernel(EncArgs a)
{
    static __shared__ SplitLds W;
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    PhaseProf P;
    P.init(a.prof);
    const uint32_t n = a.sampleCounts[c];
    uint32_t* sz = a.sizes + g * kStreams;
    if (n > kPassSamples) {  // the large-chunk pass takes it (or reports it unsupported)
        if (lane_id() == 0) {
            sz[0] = ~0u;
            a.status[c] = PGN_ERR_UNSUPPORTED;
            a.outSizes[c] = 0;
        }
        return;
    }
    uint8_t* base = a.streams + g * kChunkStreamBytes;
    C5Streams st{base + stream_off(0), base + stream_off(1), base + stream_off(2), base + stream_off(3), base + stream_off(4)};
    uint32_t sizes[5];
    c5_split_wave(a.samples + a.sampleOffsets[c], n, st, sizes, W);
    if (lane_id() == 0)
        for (int s = 0; s < kStreams; s++) sz[s] = sizes[s];
    P.mark(0);
    P.flush();
}

// Decoupled look-back between the single-wave range workgroups of one chunk (small batches): a
// range publishes a tagged 64-bit word (this call's epoch in bits 48..63) and later ranges wait for
// the words of the ranges before them; a workgroup only waits on lower-numbered ones, which the
// dispatcher started first.
__device__ __forceinline__ void lb_publish(uint64_t* w, uint64_t epoch, uint64_t payload)
{
    __hip_atomic_store(w, (epoch << 48) | payload, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// lane v < nv waits for word v * 3 + k of the chunk's look-back array; returns its payload (0 for v >= nv)
__device__ __forceinline__ uint64_t lb_wait(uint64_t* lb, int k, uint32_t nv, uint64_t epoch)
{
    const uint32_t v = (uint32_t)lane_id();
    uint64_t x = 0;
    if (v < nv) {
        while (true) {
            x = __hip_atomic_load(lb + 3 * v + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if ((x >> 48) == epoch) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return x & 0xFFFFFFFFFFFFull;
}
// Small batches, many CUs per chunk: the split over kSplitRanges single-wave range workgroups.
// Each publishes its class counts, sums those of the ranges before it (its places in the S / M /
// class-3 streams), splits its range and publishes the nibbles the S bytes it shares need; the last
// range writes those bytes and the stream sizes.  Same bytes as enc_split_kernel.
constexpr int kSplitRanges = 32;
__global__ __launch_bounds__(64) void enc_split_lb_kernel(EncArgs a)
{
    const size_t g = blockIdx.x / kSplitRanges;
    const uint32_t r = blockIdx.x % kSplitRanges;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    __shared__ SplitLds W;
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t n = a.sampleCounts[c];
    uint32_t* sz = a.sizes + g * kStreams;
    if (n > kPassSamples) {  // the large-chunk pass takes it
        if (r == 0 && lane == 0) {
            sz[0] = ~0u;
            a.status[c] = PGN_ERR_UNSUPPORTED;
            a.outSizes[c] = 0;
        }
        return;
    }
    uint64_t* lb = a.lookback + g * (3 * kSplitRanges);
    const uint64_t ep = a.epoch;
    const int16_t* x = a.samples + a.sampleOffsets[c];
    uint8_t* base = a.streams + g * kChunkStreamBytes;
    const C5Streams st{base + stream_off(0), base + stream_off(1), base + stream_off(2), base + stream_off(3),
                       base + stream_off(4)};
    const uint32_t steps = (n + kSplitStep - 1) / kSplitStep;
    const uint32_t s0 = steps * r / kSplitRanges, s1 = steps * (r + 1) / kSplitRanges;
    const uint32_t t0 = s0 * kSplitStep, t1 = s1 * kSplitStep < n ? s1 * kSplitStep : n;
    uint32_t cS = 0, cM = 0, cL = 0;
    if (t0 < t1) c5_split_counts(x, n, t0, t1, cS, cM, cL);
    if (lane == 0) lb_publish(lb + 3 * r, ep, (uint64_t)cS | ((uint64_t)cM << 16) | ((uint64_t)cL << 32));
    const uint64_t pc = lb_wait(lb, 0, r, ep);
    const uint32_t pS = (uint32_t)wave_sum64(pc & 0xFFFFu), pM = (uint32_t)wave_sum64((pc >> 16) & 0xFFFFu),
                   pL = (uint32_t)wave_sum64(pc >> 32);
    uint32_t firstNib = 0xFFu, lastNib = 0xFFu;
    if (t0 < t1) c5_split_range(x, n, t0, t1, st, pS, pM, pL, W, firstNib, lastNib);
    if (lane == 0) lb_publish(lb + 3 * r + 1, ep, (uint64_t)(firstNib & 0xFFu) | ((uint64_t)(lastNib & 0xFFu) << 8));
    if (r != kSplitRanges - 1) return;
    // the last range: every range's counts and nibbles -> the shared S bytes, a trailing half byte, sizes
    const uint64_t cnt = lb_wait(lb, 0, kSplitRanges, ep);
    const uint64_t nb = lb_wait(lb, 1, kSplitRanges, ep);
    const uint32_t tS = (uint32_t)wave_sum64(cnt & 0xFFFFu), tM = (uint32_t)wave_sum64((cnt >> 16) & 0xFFFFu),
                   tL = (uint32_t)wave_sum64(cnt >> 32);
    const uint32_t mS = (uint32_t)(cnt & 0xFFFFu);  // lane v: range v's S count
    const uint32_t fN = (uint32_t)(nb & 0xFFu), lN = (uint32_t)((nb >> 8) & 0xFFu);
    uint32_t at = 0, lastOwner = ~0u;
    for (uint32_t v = 0; v < (uint32_t)kSplitRanges; v++) {  // wave-uniform walk over the ranges
        const uint32_t cv = readlane_u32(mS, (int)v);
        if (cv == 0) continue;
        if ((at & 1u) && lastOwner != ~0u && lane == 0)
            gst<uint8_t>(st.S + (at >> 1), (uint8_t)(readlane_u32(lN, (int)lastOwner) | (readlane_u32(fN, (int)v) << 4)));
        at += cv;
        lastOwner = v;
    }
    if ((at & 1u) && lastOwner != ~0u && lane == 0) gst<uint8_t>(st.S + (at >> 1), (uint8_t)readlane_u32(lN, (int)lastOwner));
    if (lane == 0) {
        sz[0] = (n + 3) / 4;
        sz[1] = (tS + 1) / 2;
        sz[2] = tM;
        sz[3] = tL;
        sz[4] = tL;
    }
}

constexpr size_t kSplitWgMaxChunks = 64;  // batches up to this many chunks take the small-batch kernels

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void enc_zstd_kernel(EncArgs a)
{
    const int lane = lane_id();
    const EncLayout lay = enc_layout();
    uint8_t* sbase = a.slotScratch + (size_t)blockIdx.x * a.slotBytes;
    EncScratch S;
    S.ht = (uint32_t*)(sbase + lay.ht);
    S.seqs = (z1::Seq*)(sbase + lay.seqs);
    S.codes = sbase + lay.codes;
    S.lit = sbase + lay.lit;
    S.seqSection = sbase + lay.seqSection;
    S.seqWork = (z1::SeqWork*)(sbase + lay.seqWork);
    S.maxSeq = kMaxEncSeq;
    S.huf = (uint32_t*)(sbase + lay.huf);
    S.coop = nullptr;
    uint32_t epoch = a.epochs[blockIdx.x];  // table state: epoch tag | written extent << 8 (ht_next_epoch)
    PhaseProf P;
    P.init(a.prof);
    const size_t G = a.G, units = (size_t)a.nu * G;
    while (true) {
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(a.queue, 1u);
        u = __builtin_amdgcn_readfirstlane(u);
        if (u >= units) break;
        const int s = a.nu == 1 ? 0 : unit_stream((uint32_t)(u / G));
        const size_t g = u % G;
        if (a.base + g >= a.nchunks) continue;
        const uint32_t n = a.sizes[g * kStreams + s];
        if (a.sizes[g * kStreams] == ~0u) continue;  // unsupported chunk
        ht_next_epoch(S.ht, epoch, n);
        // VBZ: the svb16 buffer starts at the offset its split recorded in sizes[1]
        const uint8_t* src = a.streams + g * kChunkStreamBytes + (a.nu == 1 ? a.sizes[g * kStreams + 1] : stream_off(s));
        uint8_t* dst = a.frames + g * kChunkFrameBytes + frame_off(s);
        const size_t fsz = zstd1_compress_wave(dst, src, n, S, epoch & 0xFFu, P);
        if (lane == 0) a.fsizes[g * kStreams + s] = (uint32_t)fsz;
        wave_sync();
    }
    if (lane == 0) a.epochs[blockIdx.x] = epoch;
    P.flush();
}

// The small-batch C5 encode places its frames itself (no enc_assemble_kernel): frame s publishes
// its size in look-back word 3 s + 2 of its chunk, waits for the sizes of frames 0 .. s-1, and
// copies itself behind their length prefixes (C5.hpp:429-462).  enc_zstd_coop_kernel numbers its
// workgroups u = s * G + g (blob order, coop_unit_stream), so every frame it waits for belongs to a
// lower-numbered workgroup, which the dispatcher started first: forward progress does not depend on
// all of a call's workgroups being resident at once (another context or process may hold CUs)
// when it fits the capacity.  Frame 4 then knows the total and writes the status, the size and the
// stats as enc_assemble_kernel does.  On DST_TOO_SMALL the bytes that fit may have been written
// (as in the fused kernel, which writes its frames straight into the blob).
__device__ __noinline__ void enc_place_frame(const EncArgs& a, size_t g, int s, const uint8_t* fr, uint32_t f)
{
    const size_t c = a.base + g;
    const int lane = lane_id();
    uint64_t* lb = a.lookback + g * (3 * kSplitRanges);
    const uint64_t ep = a.epoch;
    if (lane == 0) lb_publish(lb + 3 * s + 2, ep, f);
    const uint64_t fv = lb_wait(lb, 2, (uint32_t)s, ep);  // lane v < s: frame v's size
    const uint64_t off = wave_sum64(fv) + 8ull * (uint64_t)s;
    const uint32_t pre = s < kStreams - 1 ? 8u : 0u;
    const uint64_t cap = a.outCaps[c];
    uint8_t* out = a.out + a.outOffsets[c];
    if (off + pre + f <= cap) {
        if (pre && lane == 0) {
            const uint64_t v = f;
            __builtin_memcpy(out + off, &v, 8);
        }
        wave_copy(out + off + pre, fr, f);
    }
    if (s != kStreams - 1) return;
    const uint64_t total = off + f;
    const uint32_t* sz = a.sizes + g * kStreams;
    if (lane == 0) {
        a.status[c] = total <= cap ? PGN_OK : PGN_ERR_DST_TOO_SMALL;
        a.outSizes[c] = total;
    }
    if (a.stats && lane < kStreams) {
        a.stats[c * PGN_STATS_PER_CHUNK + lane] = sz[lane];
        a.stats[c * PGN_STATS_PER_CHUNK + 5 + lane] = lane == kStreams - 1 ? f : (uint32_t)fv;
    }
}

// Stream of unit u in the cooperative kernels: blob order (keys, S, M, Llow, Lhigh).  Not the large-
// first order of the persistent kernels: every workgroup of a cooperative launch starts at once, and
// enc_place_frame's waits must point at lower-numbered workgroups.
__device__ __forceinline__ int coop_unit_stream(uint32_t k) { return (int)k; }

// Small batches (the per-chunk calls): one workgroup of kCoopEncWaves waves per stream.  Wave 0
// compresses the stream; the histograms and the bit packing of its four-segment literals sections
// are shared with the other waves, one segment each (pgn_zenc.h CoopEncCmd).  A lone chunk's encode
// is bound by its largest stream's frame.
__global__ __launch_bounds__(64 * kCoopEncWaves) void enc_zstd_coop_kernel(EncArgs a)
{
    const int lane = lane_id();
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t G = a.G;
    const uint32_t u = blockIdx.x;
    if ((size_t)u >= (size_t)a.nu * G) return;
    const int s = a.nu == 1 ? 0 : coop_unit_stream((uint32_t)(u / G));
    const size_t g = u % G;
    if (a.base + g >= a.nchunks) return;
    if (a.sizes[g * kStreams] == ~0u) return;  // unsupported chunk (the same for every wave)
    __shared__ uint32_t winAll[(kCoopEncWaves - 1) * kWinWords];
    __shared__ CoopEncCmd cmdLds;
    lds_enc_cmd* cmd = (lds_enc_cmd*)&cmdLds;
    if (wid != 0) {
        coop_enc_helper_wave(wid, cmd, (lds_u32*)&winAll[(wid - 1) * kWinWords]);
        return;
    }
    const EncLayout lay = enc_layout();
    uint8_t* sbase = a.slotScratch + (size_t)u * a.slotBytes;
    EncScratch S;
    S.ht = (uint32_t*)(sbase + lay.ht);
    S.seqs = (z1::Seq*)(sbase + lay.seqs);
    S.codes = sbase + lay.codes;
    S.lit = sbase + lay.lit;
    S.seqSection = sbase + lay.seqSection;
    S.seqWork = (z1::SeqWork*)(sbase + lay.seqWork);
    S.maxSeq = kMaxEncSeq;
    S.huf = (uint32_t*)(sbase + lay.huf);
    S.coop = cmd;
    uint32_t epoch = a.epochs[u];  // table state of slot u (ht_next_epoch)
    PhaseProf P;
    P.init(a.prof);
    const uint32_t n = a.sizes[g * kStreams + s];
    ht_next_epoch(S.ht, epoch, n);
    const uint8_t* src = a.streams + g * kChunkStreamBytes + (a.nu == 1 ? a.sizes[g * kStreams + 1] : stream_off(s));
    uint8_t* dst = a.frames + g * kChunkFrameBytes + frame_off(s);
    const size_t fsz = zstd1_compress_wave<true>(dst, src, n, S, epoch & 0xFFu, P);
    if (lane == 0) {
        a.fsizes[g * kStreams + s] = (uint32_t)fsz;
        a.epochs[u] = epoch;
    }
    coop_enc_finish(cmd);
    if (a.lookback) enc_place_frame(a, g, s, dst, (uint32_t)fsz);  // C5 (the look-back split ran)
    P.flush();
}

__global__ __launch_bounds__(64) void enc_assemble_kernel(EncArgs a)
{
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    const int lane = lane_id();
    const uint32_t* sz = a.sizes + g * kStreams;
    if (sz[0] == ~0u) return;
    PhaseProf P;
    P.init(a.prof);
    const uint32_t* fs = a.fsizes + g * kStreams;
    uint64_t total = 0;
    for (int s = 0; s < kStreams; s++) total += (s < 4 ? 8 : 0) + fs[s];
    const uint64_t cap = a.outCaps[c];
    const bool ok = total <= cap;  // C5.hpp:420-427 "Not enough space in destination buffer"
    if (ok) {
        uint8_t* dst = a.out + a.outOffsets[c];
        const uint8_t* fr = a.frames + g * kChunkFrameBytes;
        uint64_t off = 0;
        for (int s = 0; s < kStreams; s++) {
            if (s < 4) {
                if (lane == 0) {
                    const uint64_t v = fs[s];
                    __builtin_memcpy(dst + off, &v, 8);
                }
                off += 8;
            }
            wave_copy(dst + off, fr + frame_off(s), fs[s]);
            off += fs[s];
        }
    }
    if (lane == 0) {
        a.status[c] = ok ? PGN_OK : PGN_ERR_DST_TOO_SMALL;
        a.outSizes[c] = total;
        if (a.stats) {
            for (int s = 0; s < kStreams; s++) {
                a.stats[c * PGN_STATS_PER_CHUNK + s] = sz[s];
                a.stats[c * PGN_STATS_PER_CHUNK + 5 + s] = fs[s];
            }
        }
    }
    P.mark(10);
    P.flush();
}

// ---------------------------------------------------------------------------------------------
// Decode: parse -> per-stream zstd decode -> merge
// ---------------------------------------------------------------------------------------------
struct DecUnit {
    uint64_t src;       // frame offset in the input batch
    uint32_t len;       // frame bytes
    uint32_t cs;        // frame content size (= decoded bytes expected)
    uint32_t interOff;  // offset of this stream in the chunk's intermediate
    int32_t dres;       // decoded bytes, < 0 on failure
};

struct DecArgs {
    size_t nchunks;
    const uint8_t* in;
    const uint64_t* inOffsets;
    const uint64_t* inSizes;
    int16_t* samples;
    const uint64_t* sampleOffsets;
    const uint32_t* sampleCounts;
    int32_t* status;
    DecUnit* units;      // [G][5]
    uint8_t* inter;      // G * interStride
    size_t interStride;  // bytes between chunks' intermediates: chunk_inter_bytes(capN)
    uint8_t* slotScratch;
    size_t slotBytes;
    uint32_t* queue;
    uint64_t* prof;
    size_t base, G;
    uint32_t nu;         // zstd work units per chunk: 5 (C5) or 1 (VBZ)
    uint32_t capN;       // fused kernels: as EncArgs
    const uint32_t* list;
    uint64_t* lookback;  // small batches: the range merge's published counts / sums / results (kMergeRanges x 3 per chunk)
    uint64_t epoch;      // this call's tag in those words (bits 48..63)
    uint32_t coopParse;  // dec_zstd_coop_kernel parses the chunks itself (no dec_parse_kernel launch)
    uint8_t* jobs;       // [G][5] HufJob records (pgn_hufjob.h): dec_zstd_kernel defers, dec_huf_kernel decodes; null = in place
    uint32_t hufPrio;    // dec_huf_kernel waves at raised priority (the last deferred pass: the decode's drain)
    uint64_t interBytes; // dec_chunk_kernel's claims pass: the slot intermediate's bytes (0: inter_cap(capN))
};

// The status of a chunk whose frames claim more content (ZSTD_getFrameContentSize) than the
// decoder's intermediate holds.  The reference allocates the sum of the claims (a size_t sum,
// C5.hpp:575-583) and decompresses each frame into exactly its claim (C5.hpp:588-667): a sum above
// 2^40 bytes is taken as that allocation failing (PGN_ERR_ALLOC, as the oracle), a frame whose blocks
// cannot produce its claim fails in ZSTD_decompress ("failed to decompress", PGN_ERR_ZSTD_DECOMPRESS,
// z1::frame_content_bound); only frames that could really expand that far are PGN_ERR_UNSUPPORTED.
__device__ inline int over_claim_status(const uint8_t* in, const DecUnit* u, const uint64_t* cs, int nf)
{
    uint64_t tot = 0;  // each claim capped just above the limit: five claims near 2^64 cannot wrap below it
    for (int s = 0; s < nf; s++) tot += cs[s] <= kAllocLimit ? cs[s] : kAllocLimit + 1;
    if (tot > kAllocLimit) return PGN_ERR_ALLOC;
    for (int s = 0; s < nf; s++) {
        const int64_t b = z1::frame_content_bound(in + u[s].src, (size_t)u[s].len);
        if (b < 0 || (uint64_t)b < cs[s]) return PGN_ERR_ZSTD_DECOMPRESS;
    }
    return PGN_ERR_UNSUPPORTED;
}

// The claims pass (launch_claims_decode) decodes the chunks over_claim_status leaves UNSUPPORTED, as
// the reference does: every frame into exactly its claim, in an intermediate of the claims' sum.  A
// chunk whose sum exceeds kClaimPassMax gets PGN_ERR_ALLOC (that intermediate does not fit the
// device's budget, the reference's allocation failing) -- only a blob built to expand (its blocks'
// bound is at most 32,768 times its length) reaches it.
constexpr uint64_t kClaimPassMax = (uint64_t)1 << 30;

// A blob of nf frames behind nf - 1 eight-byte length prefixes (C5.hpp:530-586; the variants'
// decompress_signal_* the same with fewer frames): false when it does not parse that far (the
// decoders' PGN_ERR_CORRUPT / PGN_ERR_NOT_ZSTD); else the claims' sum and largest claim, and
// *expand = the claims sum to at most 2^40 and every frame's blocks could produce its claim
// (z1::frame_content_bound) -- the chunks over_claim_status calls UNSUPPORTED when they exceed a
// decoder's buffer.
__host__ __device__ inline bool blob_claims(const uint8_t* src, uint64_t len, int nf, uint64_t* sum, uint64_t* maxClaim,
                                            bool* expand)
{
    uint64_t pos = 0, tot = 0, mx = 0, fo[kStreams], fl[kStreams], cs[kStreams];
    for (int s = 0; s < nf; s++) {
        uint64_t l;
        if (s < nf - 1) {
            if (pos > len || len - pos < 8) return false;
            memcpy(&l, src + pos, 8);
            pos += 8;
            if (l > len - pos) return false;
        } else {
            l = len - pos;
        }
        bool ok = false;
        cs[s] = z1::frame_content_size(src + pos, (size_t)l, &ok);
        if (!ok) return false;
        fo[s] = pos;
        fl[s] = l;
        tot += cs[s] <= kAllocLimit ? cs[s] : kAllocLimit + 1;  // capped: five claims cannot wrap
        mx = cs[s] > mx ? cs[s] : mx;
        pos += l;
    }
    bool ex = tot <= kAllocLimit;
    for (int s = 0; ex && s < nf; s++) {
        const int64_t b = z1::frame_content_bound(src + fo[s], (size_t)fl[s]);
        ex = b >= 0 && (uint64_t)b >= cs[s];
    }
    *sum = tot;
    *maxClaim = mx;
    *expand = ex;
    return true;
}
// a chunk of n samples the claims pass must decode: its frames claim more than any decoder buffer
// spaced for n samples holds (inter_cap(n) less the VBZ padding, or one frame above n bytes: the C5
// per-stream bound) and could really produce it
__host__ __device__ inline bool claims_pass_chunk(const uint8_t* src, uint64_t len, int nf, uint32_t n, uint64_t* sum)
{
    uint64_t mx = 0;
    bool ex = false;
    if (!blob_claims(src, len, nf, sum, &mx, &ex) || !ex) return false;
    return *sum + kVbzPadding > inter_cap(n) || mx > n;
}

// Unhinted batch decodes: the chunks for the claims pass, listed on the scan stream beside the
// batched pass (hdr[4] count, hdr[5] the largest claims' sum in KiB, capped at 2^32 - 1).
__global__ void claim_scan_kernel(const uint8_t* in, const uint64_t* inOffsets, const uint64_t* inSizes,
                                  const uint32_t* counts, size_t n, int nf, uint32_t* list, uint32_t* hdr)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t sum = 0;
        if (!claims_pass_chunk(in + inOffsets[i], inSizes[i], nf, counts[i], &sum)) continue;
        list[atomicAdd(hdr + 4, 1u)] = (uint32_t)i;
        const uint64_t kib = (sum + 1023) >> 10;
        atomicMax(hdr + 5, kib < 0xFFFFFFFFull ? (uint32_t)kib : 0xFFFFFFFFu);
    }
}

// one thread per chunk: the four length prefixes and the five frame headers (C5.hpp:530-586).
// Frames claiming more content than the intermediate holds (inter_cap(capN) = 2.25 capN + 1,024
// bytes, capN >= every chunk of the call), or one frame more than kPassSamples bytes, get
// over_claim_status.
__device__ inline int c5_parse_chunk(const uint8_t* in, uint64_t src0, uint64_t len, DecUnit* u, size_t interCap)
{
    const uint8_t* src = in + src0;
    uint64_t pos = 0;
    uint64_t cs[5];
    for (int s = 0; s < kStreams; s++) {
        uint64_t fl;
        if (s < 4) {
            if (pos > len || len - pos < 8) return PGN_ERR_CORRUPT;
            fl = ld64u(src + pos);
            pos += 8;
            if (fl > len - pos) return PGN_ERR_CORRUPT;
        } else {
            fl = len - pos;  // last frame length is implicit (C5.hpp:560)
        }
        bool ok = false;
        cs[s] = z1::frame_content_size(src + pos, (size_t)fl, &ok);
        if (!ok) return PGN_ERR_NOT_ZSTD;
        u[s].src = src0 + pos;
        u[s].len = (uint32_t)fl;
        pos += fl;
    }
    uint64_t off = 0;
    for (int s = 0; s < kStreams; s++) {
        if (cs[s] > kPassSamples || cs[s] > interCap - off) return over_claim_status(in, u, cs, kStreams);
        u[s].cs = (uint32_t)cs[s];
        u[s].interOff = (uint32_t)off;
        off += cs[s];
    }
    return PGN_OK;
}

__global__ __launch_bounds__(64) void dec_parse_kernel(DecArgs a)
{
    const size_t g = (size_t)blockIdx.x * 64 + lane_id();
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    // a chunk above kPassSamples is left to the large-chunk pass
    a.status[c] = a.sampleCounts[c] > kPassSamples ? PGN_ERR_UNSUPPORTED
                                                   : c5_parse_chunk(a.in, a.inOffsets[c], a.inSizes[c], a.units + g * kStreams,
                                                                    inter_cap(a.capN));
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void dec_zstd_kernel(DecArgs a)
{
    const int lane = lane_id();
    const DecLayout lay = dec_layout();
    uint8_t* sbase = a.slotScratch + (size_t)blockIdx.x * a.slotBytes;
    DecScratch S;
    S.lit = sbase + lay.lit;
    S.seqs = (uint32_t*)(sbase + lay.seqs);
    S.maxSeq = kMaxDecSeq;
    S.tables = (uint32_t*)(sbase + lay.tables);
    S.htab = (uint16_t*)(sbase + lay.htab);
    S.coopCmd = nullptr;
    S.coopStg = nullptr;
    PhaseProf P;
    P.init(a.prof);
    const size_t G = a.G, units = (size_t)a.nu * G;
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(a.queue, 1u);
    while (true) {
        const uint32_t u = __builtin_amdgcn_readfirstlane(tk);
        if (u >= units) break;
        if (lane == 0) tk = atomicAdd(a.queue, 1u);
        const int s = a.nu == 1 ? 0 : unit_stream((uint32_t)(u / G));
        const size_t g = u % G;
        const size_t c = a.base + g;
        S.job = a.jobs ? a.jobs + (g * kStreams + (size_t)s) * kJobBytes : nullptr;
        if (S.job && lane == 0) gst<uint32_t>(&((HufJob*)S.job)->flag, 0u);  // every unit of the pass: fresh
        if (c >= a.nchunks || a.status[c] != PGN_OK) continue;
        DecUnit& d = a.units[g * kStreams + s];
        // destination capacity: the frame content size (C5.hpp:588-667 sizes each stream's slot
        // exactly); VBZ's intermediate carries svb16's 16 padding bytes (signal_compression.cpp:112-118)
        const size_t cap = a.nu == 1 ? (size_t)d.cs + kVbzPadding : (size_t)d.cs;
        uint8_t* const dst = a.inter + g * a.interStride + d.interOff;
        // (the record's fields are read again for the call: kept live across the fast path they
        // pushed this kernel from 37 to 186 spilled VGPRs)
        P.mark(3);
        long r = dec_frame_fast(a.in + d.src, d.len, dst, cap, S.job, S.htab, P, sDec.hb);
        P.mark(2);  // (phase 2: the fast path, or its fall-through)
        if (r < 0) r = zstd_decompress_wave(a.in + d.src, d.len, dst, cap, S, P);
        if (lane == 0) d.dres = (int32_t)r;
        wave_sync();
    }
    P.flush();
}

// ---------------------------------------------------------------------------------------------
// Deferred four-stream Huffman sections (pgn_hufjob.h): one lane per stream, kHufFrames frames per
// wave (lane 4f + k: stream k of frame f).  The wave takes the frames of one stream type (M, keys,
// ...) of kHufFrames consecutive chunks, so its lanes' streams have nearly the same length.  The
// compact tables go to LDS; a lane keeps a 64-bit left-aligned bit container: a symbol is a peek of
// the top bits, the compact-table read, a 64-bit shift by the code length (the entry's low byte) and
// the symbol byte packed four to a word; every second symbol the container takes the next dword when
// it holds 32 bits or fewer (a code is at most 11 bits, so two symbols always fit).
//
// Memory pattern (what the loop is built around; measured: tools/gpu_k2diag.sh).
// * On gfx9 one counter (vmcnt) covers loads and stores and retires in order, so waiting for a load
//   also waits for every store issued before it.  The loop issues the same memory operations every
//   iteration, unconditionally (nothing is branched around): two 16-byte loads per 16-symbol
//   iteration, consumed at the start of the next one.
// * Input: the stream is read backwards in 16-byte blocks (block b at gtop - 16 b); dword j of block
//   b sits at ring position 4 b + 3 - j of the lane's 16-dword LDS ring ([slot][lane],
//   conflict-free), so block b is ring group b & 3.  An iteration consumes at most 176 bits (six
//   dwords), so loading blocks bc + 2 and bc + 3 (bc: the block of the next dword) one iteration
//   ahead always covers the next iteration and overwrites only consumed groups.
// * Output: whole 128-byte lines.  A lane's 16-byte output blocks (each joins the previous and the
//   current iteration's words with v_alignbyte, for any destination alignment) written one per
//   iteration left 64 partial lines per wave open in L2; evicted half-written, they cost more than
//   the decode (2.84 -> 1.63 ms per 20,000 chunks with the stores sent to one line).  So every lane
//   starts 7 - m0 iterations late, m0 being its blocks before its first 128-byte boundary, and after
//   an 8-iteration prologue (those blocks stored one by one) all lanes' lines end on the same
//   iterations: the main loop runs trips of 8 iterations and stores each lane's line as 8
//   consecutive 16-byte stores at the trip's end.
// * Lanes outside their stream's iterations are frozen: their peek reads a 16-entry zero table (code
//   length 0), their stores go to a junk line, their loads stay inside their stream.
// The head and tail bytes are byte stores.  After its symbols a stream must end exactly at its first
// bit (the strict rule of huf_decode4_wave), else the frame's result is kDecErrHufStream.
// ---------------------------------------------------------------------------------------------
constexpr int kHufFrames = 16;
#ifndef PGN_K2_PF
#define PGN_K2_PF 1
#endif
constexpr uint32_t kPf = PGN_K2_PF;             // iterations between a block load and its staging
constexpr uint32_t kRing = 16 * kPf;            // dwords per lane (4 kPf blocks)
constexpr uint32_t kRingBlocks = kRing / 4;
constexpr uint32_t kTabStride = kJobTabUse;     // LDS table entries per frame
constexpr uint32_t kZeroTab = 16;               // frozen lanes' table entries
constexpr size_t kHufJunkBytes = 64 * 128;      // frozen lanes' store target: a line per lane, shared by all waves
static_assert((2 * kTabStride) % 16 == 0, "frame tables stay 16-byte aligned");

__device__ __forceinline__ uint64_t shl64(uint64_t c, uint32_t e)  // c << (e & 63), one v_lshlrev_b64
{
    return c << (e & 63u);
}
__device__ __forceinline__ uint32_t cnd(bool c, uint32_t a, uint32_t b)  // c ? a : b, one v_cndmask
{
    uint32_t r;
    asm volatile("v_cndmask_b32 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"((uint64_t)ballot(c)));
    return r;
}
__device__ __forceinline__ uint32_t pick4(bool q1, bool q2, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return cnd(q2, cnd(q1, d, c), cnd(q1, b, a));
}
__device__ __forceinline__ uint32_t sel4(const uint4& v, uint32_t i)
{
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

__global__ __launch_bounds__(64) void dec_huf_kernel(DecArgs a)
{
    __shared__ __attribute__((aligned(16))) uint16_t tabs[kHufFrames * kTabStride + kZeroTab];
    __shared__ uint32_t ring[kRing * 64];
    const uint32_t lane = (uint32_t)lane_id();
    const size_t G = a.G;
    const uint32_t ngrp = (uint32_t)((G + kHufFrames - 1) / kHufFrames);
    const uint32_t kq = blockIdx.x / ngrp;  // queue position: the large streams' groups first
    if (kq >= a.nu) return;
    const int s = unit_stream(kq);
    const size_t g0 = (size_t)(blockIdx.x % ngrp) * kHufFrames;
    const uint32_t f = lane >> 2, q = lane & 3;
    const size_t g = g0 + f;
    const bool inb = g < G && a.base + g < a.nchunks;
    const HufJob* J = (const HufJob*)(a.jobs + (inb ? (g * kStreams + (size_t)s) * kJobBytes : 0));
    const uint32_t flag = inb ? gld<uint32_t>(&J->flag) : 0u;
    const uint64_t fm = ballot(flag != 0);
    if (fm == 0) return;
    if (a.hufPrio) __builtin_amdgcn_s_setprio(3);  // ahead of the merges sharing the CU (the drain)
    // phase profile build: dec_huf's own region of the profile buffer (kHufProfOff, DecArgs.prof = +kPhases)
    PhaseProf Pp;
    Pp.init(a.prof ? a.prof + (kHufProfOff - kPhases) : nullptr);
    Pp.count(0);
    Pp.count(2, (uint64_t)__builtin_popcountll(fm));
    // the pending frames' compact tables (kTabStride entries each, 16 bytes per lane; all loads in
    // flight at once)
    {
        const uint32_t lt = lane < kTabStride / 8 ? lane : kTabStride / 8 - 1;
        uint4 tv[kHufFrames];
#pragma unroll
        for (int ff = 0; ff < kHufFrames; ff++) {
            const size_t gf = (fm >> (4 * ff)) & 1u ? g0 + (size_t)ff : g0;
            tv[ff] = gld<uint4>(a.jobs + (gf * kStreams + (size_t)s) * kJobBytes + sizeof(HufJob) + 16 * lt);
        }
#pragma unroll
        for (int ff = 0; ff < kHufFrames; ff++)
            if (lane < kTabStride / 8) *(uint4*)&tabs[ff * kTabStride + 8 * lane] = tv[ff];
        if (lane < kZeroTab / 2) ((uint32_t*)&tabs[kHufFrames * kTabStride])[lane] = 0u;
    }
    uint8_t* const junk = a.jobs + G * kStreams * kJobBytes + 128 * lane;
    Pp.mark(0);  // the job flags and the compact tables in LDS
    // this lane's stream
    uint64_t hp = 0, dstp = 0;
    uint4 len = make_uint4(0, 0, 0, 0), prm = make_uint4(0, 11, 0, 0);
    uint32_t C2 = 0;
    if (flag) {
        hp = gld<uint64_t>(&J->hp);
        dstp = gld<uint64_t>(&J->dst);
        len = gld<uint4>(&J->len[0]);
        prm = gld<uint4>(&J->rs);
        C2 = gld<uint32_t>(&J->C2);
    }
    const uint32_t rs = prm.x, tl = prm.y, d1 = prm.z & 0xFFu, d2 = prm.z >> 8, C1 = prm.w;
    const uint32_t so = (q > 0 ? len.x : 0u) + (q > 1 ? len.y : 0u) + (q > 2 ? len.z : 0u);
    const uint32_t sl = sel4(len, q);
    const uint32_t seg = (rs + 3) / 4;
    uint32_t nsym = flag ? (q == 3 ? rs - 3 * seg : seg) : 0u;
    const uint8_t* src = (const uint8_t*)hp + 6 + so;
    uint8_t* sdst = (uint8_t*)dstp + (size_t)seg * q;
    const uint32_t lastB = (flag && sl) ? (uint32_t)gb(src + sl - 1) : 0u;
    bool bad = flag && lastB == 0;
    const bool live = flag && !bad;
    if (!live) nsym = 0;
    const uint32_t sh1 = 32 - tl, shA = sh1 + d1, shB = sh1 + d2;
    // ---- bit reader.  Lanes without a stream read their junk line (readable, never decoded).
    const uint64_t e = live ? (uint64_t)src + sl - 1 : (uint64_t)junk;
    const uint64_t amin = live ? ((uint64_t)src & ~(uint64_t)15) : (uint64_t)junk;  // blocks holding stream bytes
    const uint64_t gtop = e & ~(uint64_t)15;
    const uint32_t bmax = (uint32_t)((gtop - amin) >> 4);
#if PGN_K2_DIAG == 2  // diagnostic (wrong output): every block load reads the stream's top block
    auto blk = [&](uint32_t b) { return gld<uint4>((const void*)(gtop - 16ull * (b < bmax ? b : bmax) * 0)); };
#else
    auto blk = [&](uint32_t b) { return gld<uint4>((const void*)(gtop - 16ull * (b < bmax ? b : bmax))); };
#endif
    auto stage = [&](uint32_t b, const uint4& v) {  // block b -> ring group b % kRingBlocks (highest address first)
        uint32_t* r = ring + lane + 256u * (b & (kRingBlocks - 1u));
        r[0] = v.w;
        r[64] = v.z;
        r[128] = v.y;
        r[192] = v.x;
    };
    const uint32_t hb = lastB ? z1::highbit32(lastB) : 0u;
    const uint32_t i0 = (uint32_t)(e >> 2) & 3u;
    const uint32_t v0 = live ? (uint32_t)(e & 3u) * 8u + hb : 0u;  // valid bits of the top dword
    const uint32_t totalBits = sl ? (sl - 1) * 8u + hb : 0u;
    const uint32_t ins0 = 4 - i0;  // ring position of the dword below the top one
    // insb: the ring position of the next dword times 256 (its slot's byte offset in the ring, before
    // the wrap), so a refill advances it and forms the LDS address with one instruction each
    uint32_t insb = ins0 << 8, avail = v0;
    const uint32_t laneOff = 4u * lane;
    auto ring_at = [&](uint32_t ib) -> uint32_t {  // ring[64 * ((ib >> 8) & (kRing - 1)) + lane]
        return *(const uint32_t*)((const uint8_t*)ring + ((ib & ((kRing - 1) << 8)) | laneOff));
    };
    uint64_t C;
    uint32_t nd;
    // blocks in flight: slot 0 was loaded kPf iterations ago (staged next), slot kPf - 1 last
    uint4 La[kPf], Lb[kPf];
    uint32_t lb[kPf];  // block of La (Lb: lb + 1)
    auto issue = [&](uint32_t slot) {
        lb[slot] = (insb >> 10) + 2 * kPf;
        La[slot] = blk(lb[slot]);
        Lb[slot] = blk(lb[slot] + 1);
    };
    {
        uint4 b0v[2 * kPf + 2];
#pragma unroll
        for (uint32_t k = 0; k < 2 * kPf + 2; k++) b0v[k] = blk(k);
#pragma unroll
        for (uint32_t k = 0; k < kPf; k++) {  // the loop's pattern: two loads, then one store
            issue(k);
            gst<uint4>(junk, make_uint4(0, 0, 0, 0));
        }
#pragma unroll
        for (uint32_t k = 0; k < 2 * kPf + 2; k++) stage(k, b0v[k]);
        const uint4 b0 = b0v[0];
        const uint32_t dw0 = sel4(b0, i0);
        C = v0 ? ((uint64_t)dw0 << (64 - v0)) : 0ull;
        // first refill (avail <= 31), and a second one when the container still holds only 32
        // bits: every pair of symbols starts with at least 33
        nd = ring_at(insb);
        C |= shl64((uint64_t)nd, 32u - avail);
        avail += 32;
        insb += 256;
        nd = ring_at(insb);
        if (avail <= 32) {
            C |= (uint64_t)nd;
            avail += 32;
            insb += 256;
            nd = ring_at(insb);
        }
    }
    // refill check: the dword goes into Cadd, which the next symbol ORs into the container only
    // after its table read has been issued (its peek is valid without it: a pair of symbols starts
    // with at least 33 bits and takes at most 22), so the refill is off the symbols' latency chain
    uint64_t Cadd = 0;
    auto refill = [&]() {
        const uint32_t m01 = avail <= 32 ? 1u : 0u;
        const uint32_t x = m01 ? nd : 0u;
        Cadd = shl64((uint64_t)x, 32u - avail);
        avail += m01 << 5;  // one v_lshl_add each
        insb += m01 << 8;
        nd = ring_at(insb);
    };
    // table byte addresses: entry min(p, (p >> d1) + C1, (p >> d2) + C2) of the lane's compact table
    // (pgn_hufjob.h), p = peek >> (32 - tl); tb / tc1 / tc2 carry the table base (the zero table when
    // frozen: then every candidate is the zero table's base plus a peek shift, the smallest at most 15)
    const uint32_t tbLive = f * kTabStride, tbZero = kHufFrames * kTabStride;
    uint32_t tb = tbLive, tc1 = C1 + tbLive, tc2 = C2 + tbLive, s1 = sh1;
    auto symbol = [&](bool merge) -> uint32_t {
        const uint32_t hi = (uint32_t)(C >> 32);
        const uint32_t a0 = ((hi >> s1) + tb) << 1, a1 = ((hi >> shA) + tc1) << 1, a2 = ((hi >> shB) + tc2) << 1;
        const uint32_t am = a0 < a1 ? a0 : a1;
#if PGN_K2_DIAG == 3  // diagnostic (wrong output): the table read replaced by arithmetic on the peek
        const uint32_t ent = ((am < a2 ? am : a2) & 0xFF00u) | (4u + (hi >> 30));
#else
        const uint32_t ent = *(const uint16_t*)((const uint8_t*)tabs + (am < a2 ? am : a2));
#endif
        C = shl64(merge ? (C | Cadd) : C, ent);
        avail -= ent & 0xFFu;
        return ent;
    };
    auto word4 = [&]() -> uint32_t {  // four symbols (refill checks after the second and fourth)
        const uint32_t e0 = symbol(true);
        const uint32_t e1 = symbol(false);
        refill();
        const uint32_t e2 = symbol(true);
        const uint32_t e3 = symbol(false);
        refill();
        // byte 1 of each entry: the symbol
        return __builtin_amdgcn_perm(e1, e0, 0x0C0C0501u) | __builtin_amdgcn_perm(e3, e2, 0x05010C0Cu);
    };
    auto freeze = [&](bool fz) {  // frozen: code length 0 from the zero table (peek < 16)
        tb = fz ? tbZero : tbLive;
        tc1 = fz ? tbZero : C1 + tbLive;
        tc2 = fz ? tbZero : C2 + tbLive;
        s1 = fz ? 28u : sh1;
    };
    // ---- output geometry: block D_m = output bytes [h + 16 m, h + 16 m + 16) at A0 + 16 m (16-byte
    // aligned), made in the iteration after super-group m from its words (P) and the next one's (W)
    // at byte offset h (a funnel: dword offset h / 4 by selects, byte offset h % 4 by v_alignbyte).
    // m0 blocks precede the lane's first 128-byte boundary; the lane's super-group li runs in global
    // iteration li + 7 - m0, so D_{m0 + 8 t + k} comes out of global iteration 8 + 8 t + k.
    const uint32_t h = (16u - ((uint32_t)(uintptr_t)sdst & 15u)) & 15u;  // head bytes before the first block
    uint8_t* A0 = sdst + h;
    const uint32_t rb = h & 3u;
    const bool q1 = (h >> 2) & 1u, q2 = (h >> 3) & 1u;
    const uint32_t m0 = ((128u - ((uint32_t)(uintptr_t)A0 & 127u)) & 127u) >> 4;
    const int sft = 7 - (int)m0;
    const int sg = (int)(nsym / 16);  // super-groups of 16 symbols
    const int nD = sg - 1;            // whole blocks D_0 .. D_{sg-2}
    uint32_t P[4] = {0, 0, 0, 0}, F[4] = {0, 0, 0, 0};
    auto active = [&](int gi) { const int li = gi - sft; return li >= 0 && li < sg; };
    // one global iteration: stage the blocks loaded an iteration ago, load the next two, decode 16
    // symbols; returns block D_{li - 1}
    auto iteration = [&](int gi) -> uint4 {
        stage(lb[0], La[0]);
        stage(lb[0] + 1, Lb[0]);
#pragma unroll
        for (uint32_t k = 0; k + 1 < kPf; k++) {
            lb[k] = lb[k + 1];
            La[k] = La[k + 1];
            Lb[k] = Lb[k + 1];
        }
        issue(kPf - 1);
        uint32_t W[4];
#pragma unroll
        for (int k = 0; k < 4; k++) W[k] = word4();
        // X_m = word h / 4 + m of {P, W}: two levels of per-lane selects (no indexed array, which
        // the compiler would place in scratch)
        const uint32_t X0 = pick4(q1, q2, P[0], P[1], P[2], P[3]), X1 = pick4(q1, q2, P[1], P[2], P[3], W[0]),
                       X2 = pick4(q1, q2, P[2], P[3], W[0], W[1]), X3 = pick4(q1, q2, P[3], W[0], W[1], W[2]),
                       X4 = pick4(q1, q2, W[0], W[1], W[2], W[3]);
        const uint4 D = make_uint4(__builtin_amdgcn_alignbyte(X1, X0, rb), __builtin_amdgcn_alignbyte(X2, X1, rb),
                                   __builtin_amdgcn_alignbyte(X3, X2, rb), __builtin_amdgcn_alignbyte(X4, X3, rb));
        const bool act = active(gi);
        if (gi < 8) {  // the first super-group (li = 0) falls in the prologue: its head bytes
            const bool first = gi == sft;
#pragma unroll
            for (int k = 0; k < 4; k++) F[k] = cnd(first, W[k], F[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) P[k] = cnd(act, W[k], P[k]);
        freeze(!active(gi + 1));
        return D;
    };
    freeze(!active(0));
    // prologue: global iterations 0 .. 7, the blocks before each lane's first line one by one
    // (unrolled: the in-flight slots rotate by renaming, not by copies that would wait for the loads)
#pragma unroll
    for (int gi = 0; gi < 8; gi++) {
        const uint4 D = iteration(gi);
        const int m = gi - sft - 1;
#if PGN_K2_DIAG == 1  // diagnostic (wrong output): every store to the junk line
        uint8_t* ad = junk;
#else
        uint8_t* ad = (m >= 0 && m < nD) ? A0 + 16 * m : junk;
#endif
        gst<uint4>(ad, D);
    }
    // the trip loop's pattern: loads, then eight stores (so its first wait is on the loads only)
#pragma unroll
    for (int k = 1; k < 8; k++) gst<uint4>(junk + 16 * k, make_uint4(0, 0, 0, 0));
    // trips of 8 iterations: one whole line per lane
    const int lines = nD > (int)m0 ? (nD - (int)m0 + 7) / 8 : 0;
    const int trips = (int)wave_max((uint32_t)lines);
    Pp.mark(1);  // stream setup, first loads, the 8-iteration prologue
    Pp.count(1, (uint64_t)trips);
    Pp.count(3, (uint64_t)wave_sum(nsym));
    for (int t = 0; t < trips; t++) {
        uint4 Dk[8];
#pragma unroll
        for (int k = 0; k < 8; k++) Dk[k] = iteration(8 + 8 * t + k);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int m = (int)m0 + 8 * t + k;
#if PGN_K2_DIAG == 1
            uint8_t* ad = junk + 16 * k;
#else
            uint8_t* ad = m < nD ? A0 + 16 * m : junk + 16 * k;
#endif
            gst<uint4>(ad, Dk[k]);
        }
    }
    Pp.mark(2);  // the trips of 8 iterations
#pragma unroll
    for (uint32_t k = 0; k < kPf; k++) {
        stage(lb[k], La[k]);
        stage(lb[k] + 1, Lb[k]);
    }
    freeze(false);
    C |= Cadd;
    Cadd = 0;
    // the head bytes (in the first super-group) and the pending bytes of the last one
    if (sg > 0) {
        for (uint32_t b = 0; b < h; b++) gst<uint8_t>(sdst + b, (uint8_t)(sel4(make_uint4(F[0], F[1], F[2], F[3]), b >> 2) >> (8 * (b & 3))));
        const uint32_t J16 = 16 * (uint32_t)sg - 16;  // first symbol of the last super-group
        for (uint32_t b = h; b < 16; b++)
            gst<uint8_t>(sdst + J16 + b, (uint8_t)(sel4(make_uint4(P[0], P[1], P[2], P[3]), b >> 2) >> (8 * (b & 3))));
    }
    // the remaining symbols one by one (fewer than 16: the ring holds them)
    for (uint32_t i = 16 * (uint32_t)sg; i < nsym; i++) {
        const uint32_t ent = symbol(true);
        refill();
        gst<uint8_t>(sdst + i, (uint8_t)(ent >> 8));
    }
    // exact end: the stream's bits consumed to its first bit
    if (live) bad = (v0 + 32u * ((insb >> 8) - ins0) - avail) != totalBits;
    const uint64_t bm = ballot(bad);
    if (q == 0 && flag && ((bm >> (4 * f)) & 0xFull)) gst<int32_t>(&a.units[g * kStreams + (size_t)s].dres, (int32_t)z1::kDecErrHufStream);
    Pp.mark(3);  // drain, head / tail bytes, the last symbols, the end check
    Pp.flush();
}

// The same jobs, latency first (the last deferred pass of a call: nothing overlaps its sections
// once the frame decode has ended -- the decode's drain).  A workgroup of four waves per job, one wave
// per stream with all 64 lanes (huf_decode1of4_wave64, the cooperative decoder: speculative windows,
// a sync, an exact second pass), so a stream's ~16,000 symbols take a few 64-lane rounds instead of
// one lane's serial chain; about 2.5 times the instructions of dec_huf_kernel, on a chip that is
// otherwise waiting.  The compact table is expanded back into the full 2^tl-entry table in LDS.  Same
// symbols and the same strict end rule; a failing stream marks its frame kDecErrHufStream.
__global__ __launch_bounds__(64 * kCoopWaves) void dec_huf_wide_kernel(DecArgs a)
{
    const uint32_t u = blockIdx.x;
    const size_t G = a.G;
    if ((size_t)u >= (size_t)a.nu * G) return;
    const int s = unit_stream((uint32_t)(u / G));  // large streams first
    const size_t g = u % G;
    if (a.base + g >= a.nchunks) return;
    const HufJob* J = (const HufJob*)(a.jobs + (g * kStreams + (size_t)s) * kJobBytes);
    if (gld<uint32_t>(&J->flag) == 0) return;  // the same for every wave of the group
    __shared__ uint32_t stgAll[kCoopWaves * kCoopStgWords];
    __shared__ uint32_t bad;
    const uint32_t tid = threadIdx.x;
    const int wid = (int)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint64_t hp = gld<uint64_t>(&J->hp), dstp = gld<uint64_t>(&J->dst);
    const uint4 len = gld<uint4>(&J->len[0]);
    const uint4 prm = gld<uint4>(&J->rs);
    const uint32_t C2 = gld<uint32_t>(&J->C2);
    const uint32_t rs = prm.x, tl = prm.y, d1 = prm.z & 0xFFu, d2 = prm.z >> 8, C1 = prm.w;
    // the full table from the compact one: entry min(p, (p >> d1) + C1, (p >> d2) + C2), swapped back
    // to symbol | nbBits << 8
    const uint16_t* ct = (const uint16_t*)(a.jobs + (g * kStreams + (size_t)s) * kJobBytes + sizeof(HufJob));
    for (uint32_t p = tid; p < (1u << tl); p += 64 * kCoopWaves) {
        const uint32_t i1 = (p >> d1) + C1, i2 = (p >> d2) + C2;
        uint32_t i = p < i1 ? p : i1;
        i = i < i2 ? i : i2;
        const uint32_t c = gld<uint16_t>(ct + i);
        sDec.tab[p] = (uint16_t)((c >> 8) | ((c & 0xFFu) << 8));
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    PhaseProf P;
    P.init(nullptr);
    const size_t remain = 6 + (size_t)len.x + len.y + len.z + len.w;
    const bool ok = huf_decode1of4_wave64(tl, (const uint8_t*)hp, remain, (uint8_t*)dstp, rs, len.x | (len.y << 16), len.z,
                                          wid, (lds_u32*)&stgAll[wid * kCoopStgWords + 2 * 64], P);
    if (!ok && lane_id() == 0) atomicOr(&bad, 1u);
    __syncthreads();
    if (tid == 0 && bad) gst<int32_t>(&a.units[g * kStreams + (size_t)s].dres, (int32_t)z1::kDecErrHufStream);
}

// Small batches (the per-chunk calls): one workgroup of kCoopWaves waves per work unit.  Wave 0
// decodes the frame; the four Huffman streams of each literals section are decoded by the four
// waves at once, 64 lanes per stream (pgn_zdec.h CoopCmd).  A lone 100,000-sample chunk's decode
// is bound by its largest frame's Huffman rounds, which this cuts about fourfold.
constexpr size_t kCoopMaxChunks = 64;  // batches up to this many chunks use it
__global__ __launch_bounds__(64 * kCoopWaves) void dec_zstd_coop_kernel(DecArgs a)
{
    const int lane = lane_id();
    const int wid = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t G = a.G;
    const uint32_t u = blockIdx.x;
    if ((size_t)u >= (size_t)a.nu * G) return;
    const int s = a.nu == 1 ? 0 : unit_stream((uint32_t)(u / G));
    const size_t g = u % G;
    const size_t c = a.base + g;
    if (c >= a.nchunks) return;
    __shared__ int32_t parseRc;
    __shared__ DecUnit myUnit;
    if (a.coopParse) {  // the chunk's prefixes and frame headers (dec_parse_kernel's work), here
        if (threadIdx.x == 0) {
            DecUnit uu[kStreams];
            const int rc = a.sampleCounts[c] > kPassSamples ? PGN_ERR_UNSUPPORTED
                                                            : c5_parse_chunk(a.in, a.inOffsets[c], a.inSizes[c], uu,
                                                                             inter_cap(a.capN));
            parseRc = rc;
            if (rc == PGN_OK) myUnit = uu[s];
            if (s == 0) {  // the chunk's first frame publishes its status and frame records for the merge
                a.status[c] = rc;
                if (rc == PGN_OK) {
                    for (int k = 0; k < kStreams; k++) {
                        DecUnit& w = a.units[g * kStreams + k];
                        w.src = uu[k].src;
                        w.len = uu[k].len;
                        w.cs = uu[k].cs;
                        w.interOff = uu[k].interOff;
                    }
                }
            }
        }
        __syncthreads();
        if (parseRc != PGN_OK) return;  // the same for every wave of the group
    } else {
        if (a.status[c] != PGN_OK) return;
        if (threadIdx.x == 0) myUnit = a.units[g * kStreams + s];
        __syncthreads();
    }
    PhaseProf P;
    P.init(a.prof);
    __shared__ uint32_t stgAll[kCoopWaves * kCoopStgWords];
    __shared__ CoopCmd cmdLds;
    lds_cmd* cmd = (lds_cmd*)&cmdLds;
    lds_u32* stg = (lds_u32*)&stgAll[wid * kCoopStgWords + 2 * 64];
    if (wid != 0) {
        coop_helper_wave(wid, cmd, stg, P);
        P.flush();
        return;
    }
    const DecLayout lay = dec_layout();
    uint8_t* sbase = a.slotScratch + (size_t)u * a.slotBytes;
    DecScratch S;
    S.lit = sbase + lay.lit;
    S.seqs = (uint32_t*)(sbase + lay.seqs);
    S.maxSeq = kMaxDecSeq;
    S.tables = (uint32_t*)(sbase + lay.tables);
    S.htab = (uint16_t*)(sbase + lay.htab);
    S.coopCmd = cmd;
    S.coopStg = stg;
    S.job = nullptr;
    const uint64_t dsrc = myUnit.src;
    const uint32_t dlen = myUnit.len, dcs = myUnit.cs, doff = myUnit.interOff;
    const size_t cap = a.nu == 1 ? (size_t)dcs + kVbzPadding : (size_t)dcs;
    const long r = zstd_decompress_wave<true>(a.in + dsrc, dlen, a.inter + g * a.interStride + doff, cap, S, P);
    if (lane == 0) a.units[g * kStreams + s].dres = (int32_t)r;
    coop_finish(cmd);
    P.flush();
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void dec_merge_kernel(DecArgs a)
{
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    if (a.status[c] != PGN_OK) return;
    static __shared__ MergeLds W;
    PhaseProf P;
    P.init(a.prof);
#if PGN_MERGE_DIAG == 1  // diagnostic: chunk g merges chunk g % 32's intermediate (L2-resident reads, same work on equal-size chunks)
    const size_t gi = g % 32;
#else
    const size_t gi = g;
#endif
    const DecUnit* d = a.units + gi * kStreams;
    uint64_t total = 0;
    int st = PGN_OK;
    for (int s = 0; s < kStreams; s++) {
        if (d[s].dres < 0) st = PGN_ERR_ZSTD_DECOMPRESS;
        total += d[s].cs;
    }
    if (st == PGN_OK) {
        uint64_t consumed = 0;
        const int bad = c5_merge_wave(a.inter + gi * a.interStride, total, (uint64_t)d[1].dres, (uint64_t)d[2].dres,
                                      (uint64_t)d[3].dres, a.samples + a.sampleOffsets[c], a.sampleCounts[c], &consumed, W);
        if (bad) st = PGN_ERR_CORRUPT;
        else if (consumed != total) st = PGN_ERR_REMAINING;
    }
    if (lane_id() == 0) a.status[c] = st;
    P.mark(6);
    P.flush();
}

constexpr size_t kMergeWgMaxChunks = 64;  // batches up to this many chunks take the small-batch kernels

// Small batches, many CUs per chunk: the chunk's steps in kMergeRanges ranges, one single-wave
// workgroup each, so a lone chunk's merge runs on kMergeRanges CUs instead of one.  The ranges find
// their places without another launch: each publishes its class counts, then (after summing those of
// the ranges before it) the delta sum of its stream bytes, then its result, as tagged 64-bit words
// (this call's epoch in bits 48..63) that later ranges wait for -- decoupled look-back; a workgroup
// only waits on lower-numbered ones, which the dispatcher started first.  The last range sets the
// status once every range is done.  Same bytes and statuses as dec_merge_kernel.
constexpr int kMergeRanges = 32;
__global__ __launch_bounds__(64) void dec_merge_lb_kernel(DecArgs a)
{
    const size_t g = blockIdx.x / kMergeRanges;
    const uint32_t r = blockIdx.x % kMergeRanges;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    if (a.status[c] != PGN_OK) return;
    const uint32_t lane = (uint32_t)lane_id();
#if PGN_MERGE_DIAG == 1  // diagnostic: chunk g merges chunk g % 32's intermediate (L2-resident reads, same work on equal-size chunks)
    const size_t gi = g % 32;
#else
    const size_t gi = g;
#endif
    const DecUnit* d = a.units + gi * kStreams;
    uint64_t total = 0;
    int st = PGN_OK;
    for (int s = 0; s < kStreams; s++) {
        if (d[s].dres < 0) st = PGN_ERR_ZSTD_DECOMPRESS;
        total += d[s].cs;
    }
    if (st != PGN_OK) {  // the same for every range of the chunk
        if (r == 0 && lane == 0) a.status[c] = st;
        return;
    }
    __shared__ MergeLds W;
    uint64_t* lb = a.lookback + g * (3 * kMergeRanges);
    const uint64_t ep = a.epoch;
    const uint32_t n = a.sampleCounts[c];
    const uint8_t* in = a.inter + g * a.interStride;
    int16_t* out = a.samples + a.sampleOffsets[c];
    const uint64_t dS = (uint64_t)d[1].dres, dM = (uint64_t)d[2].dres, dLl = (uint64_t)d[3].dres;
    const uint64_t kl = ((uint64_t)n + 3) / 4;
    const uint64_t ps = kl, pm = kl + dS, pl = kl + dS + dM, ph = kl + dS + dM + dLl;
    const uint32_t steps = (n + kSplitStep - 1) / kSplitStep;
    const uint32_t s0 = (uint32_t)((uint64_t)steps * r / kMergeRanges), s1 = (uint32_t)((uint64_t)steps * (r + 1) / kMergeRanges);
    const uint32_t t0 = s0 * kSplitStep, t1 = s1 * kSplitStep < n ? s1 * kSplitStep : n;
    // 1. own class counts (16 bits each: a range has at most 16 steps below PGN pass sizes)
    uint32_t cS = 0, cM = 0, cL = 0;
    if (kl <= total) c5_class_counts(in, n, t0, t1, cS, cM, cL);
    if (lane == 0) lb_publish(lb + 3 * r, ep, (uint64_t)cS | ((uint64_t)cM << 16) | ((uint64_t)cL << 32));
    // 2. the counts before me -> my stream spans -> my delta sum
    const uint64_t pc = lb_wait(lb, 0, r, ep);
    const uint64_t sN0 = wave_sum64(pc & 0xFFFFu), mN0 = wave_sum64((pc >> 16) & 0xFFFFu), lN0 = wave_sum64(pc >> 32);
    const uint64_t sN1 = sN0 + cS, mN1 = mN0 + cM, lN1 = lN0 + cL;
    const bool inside = kl <= total && ps + ((sN1 + 1) >> 1) <= total && pm + mN1 <= total && pl + lN1 <= total &&
                        ph + lN1 <= total;
    uint32_t sum = 0;
    if (inside) sum = c5_range_delta_sum(in, ps, pm, pl, ph, sN0, sN1, mN0, mN1, lN0, lN1);
    if (lane == 0) lb_publish(lb + 3 * r + 1, ep, (uint64_t)sum | ((uint64_t)(inside ? 0u : 1u) << 32));
    // 3. the running sum at my start: the sums before me; merge unless a range so far is outside
    const uint64_t ps_ = lb_wait(lb, 1, r, ep);
    const uint32_t carryIn = (uint32_t)wave_sum64(ps_ & 0xFFFFu);
    const bool outsideBefore = wave_sum64((ps_ >> 32) & 1u) != 0;
    int bad = (!inside || outsideBefore) ? 1 : 0;
    if (!bad) {
        uint32_t carry = carryIn;
        uint64_t lEnd = 0;
        bad = c5_merge_range<false>(in, total, dS, dM, dLl, out, n, t0, t1, sN0, mN0, lN0, carry, &lEnd, W);
    }
    if (lane == 0) lb_publish(lb + 3 * r + 2, ep, (uint64_t)(bad ? 1u : 0u));
    // 4. the last range: every range done -> status
    if (r == kMergeRanges - 1) {
        const uint64_t dn = lb_wait(lb, 2, kMergeRanges, ep);
        const bool badAny = wave_sum64(dn & 1u) != 0;
        const uint64_t lTot = lN1;  // the class-3 count through the last range
        if (lane == 0) {
            __threadfence();
            a.status[c] = badAny ? PGN_ERR_CORRUPT : ((ph + lTot != total) ? PGN_ERR_REMAINING : PGN_OK);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// VBZ (pod5::compress_signal / decompress_signal, signal_compression.cpp:37-141): split -> one
// zstd frame per chunk -> copy into place; parse -> zstd decode -> svb16 merge.  The per-chunk
// buffers are the C5 ones (a chunk's stream area holds its svb16 buffer, <= 2.125 n bytes).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void vbz_split_kernel(EncArgs a)
{
    static __shared__ VbzSplitLds W;
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    PhaseProf P;
    P.init(a.prof);
    const uint32_t n = a.sampleCounts[c];
    uint32_t* sz = a.sizes + g * kStreams;
    if (n > kPassSamples) {  // the large-chunk pass takes it
        if (lane_id() == 0) {
            sz[0] = ~0u;
            a.status[c] = PGN_ERR_UNSUPPORTED;
            a.outSizes[c] = 0;
        }
        return;
    }
    // place the buffer so that its data part (after the ceil(n/8) key bytes) is 16-byte aligned
    const uint32_t pad = (16u - (svb_key_length(n) & 15u)) & 15u;
    const uint32_t m = vbz_split_wave(a.samples + a.sampleOffsets[c], n, a.streams + g * kChunkStreamBytes + pad, W);
    if (lane_id() == 0) {
        sz[0] = m;
        sz[1] = pad;
    }
    P.mark(0);
    P.flush();
}

__global__ __launch_bounds__(64) void vbz_assemble_kernel(EncArgs a)
{
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    const int lane = lane_id();
    const uint32_t* sz = a.sizes + g * kStreams;
    if (sz[0] == ~0u) return;
    const uint32_t fs = a.fsizes[g * kStreams];
    // ZSTD_compress into the caller's span fails when the frame does not fit
    // (signal_compression.cpp:57-62 "Failed to compress data")
    const bool ok = fs <= a.outCaps[c];
    if (ok) wave_copy(a.out + a.outOffsets[c], a.frames + g * kChunkFrameBytes, fs);
    if (lane == 0) {
        a.status[c] = ok ? PGN_OK : PGN_ERR_ZSTD_COMPRESS;
        a.outSizes[c] = ok ? fs : 0;
        if (a.stats) {
            for (int s = 0; s < PGN_STATS_PER_CHUNK; s++) a.stats[c * PGN_STATS_PER_CHUNK + s] = 0;
            a.stats[c * PGN_STATS_PER_CHUNK] = sz[0];
            a.stats[c * PGN_STATS_PER_CHUNK + 5] = fs;
        }
    }
}

// one thread per chunk: ZSTD_getFrameContentSize (signal_compression.cpp:100-109)
__global__ __launch_bounds__(64) void vbz_parse_kernel(DecArgs a)
{
    const size_t g = (size_t)blockIdx.x * 64 + lane_id();
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    DecUnit* u = a.units + g * kStreams;
    bool ok = false;
    const uint64_t src0 = a.inOffsets[c], len = a.inSizes[c];
    const uint64_t cs = z1::frame_content_size(a.in + src0, (size_t)len, &ok);
    int st = PGN_OK;
    if (a.sampleCounts[c] > kPassSamples) st = PGN_ERR_UNSUPPORTED;  // the large-chunk pass takes it
    else if (!ok) st = PGN_ERR_NOT_ZSTD;
    else if (len > 0xFFFFFFFFull) st = PGN_ERR_UNSUPPORTED;
    else if (cs + kVbzPadding > inter_cap(a.capN)) {
        u->src = src0;
        u->len = (uint32_t)len;
        st = over_claim_status(a.in, u, &cs, 1);
    } else {
        u->src = src0;
        u->len = (uint32_t)len;
        u->cs = (uint32_t)cs;
        u->interOff = 0;
        u->dres = 0;
    }
    a.status[c] = st;
}

__global__ __launch_bounds__(64) void vbz_merge_kernel(DecArgs a)
{
    const size_t g = blockIdx.x;
    const size_t c = a.base + g;
    if (g >= a.G || c >= a.nchunks) return;
    if (a.status[c] != PGN_OK) return;
    static __shared__ VbzMergeLds W;
    PhaseProf P;
    P.init(a.prof);
    const DecUnit* d = a.units + g * kStreams;
    int st = PGN_OK;
    if (d->dres < 0) {
        st = PGN_ERR_ZSTD_DECOMPRESS;
    } else {
        // svb16::decode over the padded intermediate, then "consumed + padding == size"
        // (signal_compression.cpp:124-131): bytes past the content but inside the padding are the
        // "Remaining data" error, beyond it the reference reads out of bounds
        uint64_t consumed = 0;
        const uint32_t n = a.sampleCounts[c];
        const uint64_t total = (uint64_t)d->cs + kVbzPadding;
        if (svb_key_length(n) > d->cs) {  // keys alone run into the padding (or past it)
            st = svb_key_length(n) <= total ? PGN_ERR_REMAINING : PGN_ERR_CORRUPT;
        } else {
            const int bad = vbz_merge_wave(a.inter + g * a.interStride, total, a.samples + a.sampleOffsets[c], n,
                                           &consumed, W);
            if (bad) st = PGN_ERR_CORRUPT;
            else if (consumed != d->cs) st = PGN_ERR_REMAINING;
        }
    }
    if (lane_id() == 0) a.status[c] = st;
    P.mark(6);
    P.flush();
}

// ---------------------------------------------------------------------------------------------
// Fused per-chunk pipeline.  One persistent wave takes whole chunks from a queue:
//   encode: split into its slot's stream area -> the chunk's zstd frames written straight into its
//           blob behind their length prefixes -> size, status, stats;
//   decode: prefixes and frame headers -> the frames decoded into its slot's intermediate -> merge
//           into the samples, consumed-bytes check.
// Waves in different stages share each CU (VALU-bound split/merge beside latency-bound entropy
// coding), a chunk's streams are re-read by the wave that just wrote them, and frames are never
// staged and copied.  The split/merge LDS overlays the zstd stage's (stages of one wave never
// overlap in time).  Every codec runs here; C5 and VBZ also have the staged pipeline above.
// ---------------------------------------------------------------------------------------------
static_assert(sizeof(SplitLds) <= sizeof(EncLds) && sizeof(VbzSplitLds) <= sizeof(EncLds) &&
                  sizeof(Vbz0SplitLds) <= sizeof(EncLds),
              "split LDS overlay");
static_assert(sizeof(MergeLds) <= sizeof(DecLds) && sizeof(VbzMergeLds) <= sizeof(DecLds) &&
                  sizeof(Vbz0MergeLds) <= sizeof(DecLds),
              "merge LDS overlay");

// Frames per chunk: C5/C4 5, C3 4, C2 3, C1 2, VBZ/VBZ0 1 (pgnano/svb16/C*.hpp, VBZ_0.hpp)
__host__ __device__ constexpr int codec_frames(int codec)
{
    return codec == kCodecC5 || codec == kCodecC4 ? 5 : (codec == kCodecC3 ? 4 : (codec == kCodecC2 ? 3 : (codec == kCodecC1 ? 2 : 1)));
}

// slot scratch of the fused kernels for chunks of up to capN samples: the zstd scratch, then the
// chunk's streams (encode: + one frame for a stream that may not fit the destination; any one
// stream's frame, a VBZ / C1 svb16 buffer of up to ~2.13 capN the largest) or its intermediate
// (decode)
__host__ __device__ inline size_t slot_frame_bytes(uint32_t capN) { return align_up(frame_bound((size_t)capN * 9 / 4 + 64) + 64, 256); }
__host__ __device__ inline size_t enc_slot_bytes(uint32_t capN = kPassSamples)
{
    return enc_layout().bytes + chunk_stream_bytes(capN) + slot_frame_bytes(capN);
}
__host__ __device__ inline size_t dec_slot_bytes(uint32_t capN = kPassSamples) { return dec_layout().bytes + chunk_inter_bytes(capN); }

// The split and merge stages as non-inlined calls with wave-uniform arguments: each gets its own
// register allocation instead of sharing the kernel's with the state kept across the zstd calls
// (inlined, both spilled to scratch inside their step loops).
struct SplitOut {
    uint32_t s[kStreams];
};
template <bool C4>
__device__ __noinline__ SplitOut c5_split_chunk(const int16_t* x, uint32_t n, uint8_t* streams, uint32_t capN)
{
    x = uni(x);
    n = uni(n);
    streams = uni(streams);
    capN = uni(capN);
    C5Streams st{streams + stream_off(0, capN), streams + stream_off(1, capN), streams + stream_off(2, capN),
                 streams + stream_off(3, capN), streams + stream_off(4, capN)};
    SplitOut o;
    c5_split_wave<C4>(x, n, st, o.s, *reinterpret_cast<SplitLds*>(&sEnc));
    return o;
}
template <bool C3>
__device__ __noinline__ SplitOut c23_split_chunk(const int16_t* x, uint32_t n, uint8_t* streams, uint32_t capN)
{
    x = uni(x);
    n = uni(n);
    streams = uni(streams);
    capN = uni(capN);
    SplitOut o;
    c23_split_wave<C3>(x, n, streams + stream_off(0, capN), streams + stream_off(2, capN), streams + stream_off(3, capN),
                       streams + stream_off(4, capN), o.s);
    return o;
}
__device__ __noinline__ uint32_t vbz_split_chunk(const int16_t* x, uint32_t n, uint8_t* out)
{
    return vbz_split_wave(uni(x), uni(n), uni(out), *reinterpret_cast<VbzSplitLds*>(&sEnc));
}
__device__ __noinline__ uint32_t vbz0_split_chunk(const int16_t* x, uint32_t n, uint8_t* out)
{
    return vbz0_split_wave(uni(x), uni(n), uni(out), *reinterpret_cast<Vbz0SplitLds*>(&sEnc));
}
struct MergeOut {
    int bad;
    uint64_t consumed;
};
template <bool C4>
__device__ __noinline__ MergeOut c5_merge_chunk(const uint8_t* in, uint64_t total, uint64_t dS, uint64_t dM, uint64_t dLl,
                                                int16_t* out, uint32_t n)
{
    MergeOut o{0, 0};
    o.bad = c5_merge_wave<C4>(uni(in), uni(total), uni(dS), uni(dM), uni(dLl), uni(out), uni(n), &o.consumed,
                              *reinterpret_cast<MergeLds*>(&sDec));
    return o;
}
template <bool C3>
__device__ __noinline__ MergeOut c23_merge_chunk(const uint8_t* in, uint64_t total, uint64_t dA, uint64_t dB, int16_t* out,
                                                 uint32_t n)
{
    MergeOut o{0, 0};
    o.bad = c23_merge_wave<C3>(uni(in), uni(total), uni(dA), uni(dB), uni(out), uni(n), &o.consumed);
    return o;
}
__device__ __noinline__ MergeOut vbz_merge_chunk(const uint8_t* in, uint64_t total, int16_t* out, uint32_t n)
{
    MergeOut o{0, 0};
    o.bad = vbz_merge_wave(uni(in), uni(total), uni(out), uni(n), &o.consumed, *reinterpret_cast<VbzMergeLds*>(&sDec));
    return o;
}
__device__ __noinline__ MergeOut vbz0_merge_chunk(const uint8_t* in, uint64_t total, int16_t* out, uint32_t n)
{
    MergeOut o{0, 0};
    o.bad = vbz0_merge_wave(uni(in), uni(total), uni(out), uni(n), &o.consumed, *reinterpret_cast<Vbz0MergeLds*>(&sDec));
    return o;
}

__device__ __forceinline__ void enc_fail_chunk(const EncArgs& a, size_t c, int st)
{
    if (lane_id() == 0) {
        a.status[c] = st;
        a.outSizes[c] = 0;
    }
}

template <int Codec>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void enc_chunk_kernel(EncArgs a)
{
    constexpr int nf = codec_frames(Codec);
    // VBZ and VBZ0 compress straight into the destination span: a frame that does not fit fails
    // (signal_compression.cpp:57-62, VBZ_0.hpp:345-350); the multi-frame variants check the total
    // (C5.hpp:412-427) and report the required size
    constexpr bool oneFrame = nf == 1;
    const int lane = lane_id();
    const EncLayout lay = enc_layout();
    uint8_t* sbase = a.slotScratch + (size_t)blockIdx.x * a.slotBytes;
    EncScratch S;
    S.ht = (uint32_t*)(sbase + lay.ht);
    S.seqs = (z1::Seq*)(sbase + lay.seqs);
    S.codes = sbase + lay.codes;
    S.lit = sbase + lay.lit;
    S.seqSection = sbase + lay.seqSection;
    S.seqWork = (z1::SeqWork*)(sbase + lay.seqWork);
    S.maxSeq = kMaxEncSeq;
    S.huf = (uint32_t*)(sbase + lay.huf);
    S.coop = nullptr;
    const uint32_t capN = a.capN;
    uint8_t* streams = sbase + lay.bytes;
    uint8_t* fbuf = streams + chunk_stream_bytes(capN);
    uint32_t epoch = a.epochs[blockIdx.x];  // table state: epoch tag | written extent << 8 (ht_next_epoch)
    PhaseProf P;
    P.init(a.prof);
    while (true) {
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(a.queue, 1u);
        u = __builtin_amdgcn_readfirstlane(u);
        if (u >= a.nchunks) break;
        const size_t c = a.list ? a.list[u] : u;
        const uint32_t n = a.sampleCounts[c];
        if (n > capN) {  // the large-chunk pass takes it (or reports it unsupported)
            enc_fail_chunk(a, c, PGN_ERR_UNSUPPORTED);
            continue;
        }
        const int16_t* x = a.samples + a.sampleOffsets[c];
        uint32_t sz[kStreams] = {0, 0, 0, 0, 0};
        const uint8_t* src[kStreams] = {streams, streams, streams, streams, streams};
        if (Codec == kCodecVbz || Codec == kCodecC1) {
            // svb16 keys | data, the data part 16-byte aligned (as in vbz_split_kernel)
            const uint32_t pad = (16u - (svb_key_length(n) & 15u)) & 15u;
            const uint32_t m = vbz_split_chunk(x, n, streams + pad);
            src[0] = streams + pad;
            if (Codec == kCodecVbz) {
                sz[0] = m;
            } else {  // C1: the keys frame and the data frame (C1.hpp:229-266)
                sz[0] = n ? svb_key_length(n) : 0u;
                sz[1] = m - sz[0];
                src[1] = src[0] + sz[0];
            }
        } else if (Codec == kCodecVbz0) {
            sz[0] = vbz0_split_chunk(x, n, streams);
        } else if (Codec == kCodecC2 || Codec == kCodecC3) {
            const SplitOut so = c23_split_chunk<Codec == kCodecC3>(x, n, streams, capN);
#pragma unroll
            for (int s = 0; s < kStreams; s++) sz[s] = so.s[s];
            src[0] = streams + stream_off(0, capN);
            src[1] = streams + stream_off(2, capN);
            src[2] = streams + stream_off(Codec == kCodecC3 ? 3 : 4, capN);
            src[3] = streams + stream_off(4, capN);
        } else {
            const SplitOut so = c5_split_chunk<Codec == kCodecC4>(x, n, streams, capN);
#pragma unroll
            for (int s = 0; s < kStreams; s++) {
                sz[s] = so.s[s];
                src[s] = streams + stream_off(s, capN);
            }
        }
#pragma unroll
        for (int s = 0; s < kStreams; s++) sz[s] = uni(sz[s]);
        bool big = false;  // a stream above the encoder's largest frame (not reached below the chunk limit)
#pragma unroll
        for (int s = 0; s < nf; s++) big |= sz[s] > kMaxFrameBytes;
        if (big) {
            enc_fail_chunk(a, c, PGN_ERR_UNSUPPORTED);
            continue;
        }
        P.mark(0);
        P.count(9, (n + 1023) / 1024);
        wave_sync();
        uint8_t* dst = a.out + a.outOffsets[c];
        const uint64_t cap = a.outCaps[c];
        uint64_t off = 0;
        bool ok = true;
        uint32_t fs[kStreams] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < nf; s++) {
            if (s < nf - 1) off += 8;  // length prefixes of all frames but the last (C5.hpp:429-462)
            ht_next_epoch(S.ht, epoch, sz[s]);
            // straight into the blob when the frame bound fits the capacity; otherwise through the
            // slot's frame buffer (the reference compresses into its own buffers, then checks)
            const bool direct = ok && off + frame_bound(sz[s]) <= cap;
            const size_t f = uni(zstd1_compress_wave(direct ? dst + off : fbuf, src[s], sz[s], S, epoch & 0xFFu, P));
            wave_sync();
            if (!direct && ok) {
                if (off + f <= cap) wave_copy(dst + off, fbuf, f);
                else ok = false;
                wave_sync();
            }
            if (s < nf - 1 && ok && lane == 0) {
                const uint64_t v = f;
                __builtin_memcpy(dst + off - 8, &v, 8);
            }
            fs[s] = (uint32_t)f;
            off += f;
        }
        P.mark(10);
        if (lane == 0) {
            if (oneFrame) {
                a.status[c] = ok ? PGN_OK : PGN_ERR_ZSTD_COMPRESS;
                a.outSizes[c] = ok ? off : 0;
            } else {
                a.status[c] = ok ? PGN_OK : PGN_ERR_DST_TOO_SMALL;
                a.outSizes[c] = off;  // the reference's "Required size" on failure
            }
            if (a.stats) {
                for (int s = 0; s < kStreams; s++) {
                    a.stats[c * PGN_STATS_PER_CHUNK + s] = s < nf ? sz[s] : 0;
                    a.stats[c * PGN_STATS_PER_CHUNK + 5 + s] = s < nf ? fs[s] : 0;
                }
            }
        }
        wave_sync();
    }
    if (lane == 0) a.epochs[blockIdx.x] = epoch;
    P.flush();
}

// nf frames behind nf-1 length prefixes (the decompress_signal_* front half, C5.hpp:477-586):
// frame records with content sizes and intermediate offsets; the frames together must fit the
// slot's intermediate.
template <int NF>
__device__ inline int parse_frames(const uint8_t* in, uint64_t src0, uint64_t len, DecUnit* u, uint64_t* total,
                                   size_t interCap)
{
    const uint8_t* src = in + src0;
    uint64_t pos = 0, cs[kStreams];
    for (int s = 0; s < NF; s++) {
        uint64_t fl;
        if (s < NF - 1) {
            if (pos > len || len - pos < 8) return PGN_ERR_CORRUPT;
            fl = ld64u(src + pos);
            pos += 8;
            if (fl > len - pos) return PGN_ERR_CORRUPT;
        } else {
            fl = len - pos;  // the last frame's length is implicit
        }
        bool ok = false;
        cs[s] = z1::frame_content_size(src + pos, (size_t)fl, &ok);
        if (!ok) return PGN_ERR_NOT_ZSTD;
        if (fl > 0xFFFFFFFFull) return PGN_ERR_UNSUPPORTED;
        u[s].src = src0 + pos;
        u[s].len = (uint32_t)fl;
        pos += fl;
    }
    uint64_t off = 0;
    for (int s = 0; s < NF; s++) {
        if (cs[s] > interCap - kVbzPadding - off) return over_claim_status(in, u, cs, NF);
        u[s].cs = (uint32_t)cs[s];
        u[s].interOff = (uint32_t)off;
        off += cs[s];
    }
    *total = off;
    return PGN_OK;
}

template <int Codec>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void dec_chunk_kernel(DecArgs a)
{
    constexpr int nf = codec_frames(Codec);
    const int lane = lane_id();
    const DecLayout lay = dec_layout();
    uint8_t* sbase = a.slotScratch + (size_t)blockIdx.x * a.slotBytes;
    DecScratch S;
    S.lit = sbase + lay.lit;
    S.seqs = (uint32_t*)(sbase + lay.seqs);
    S.maxSeq = kMaxDecSeq;
    S.tables = (uint32_t*)(sbase + lay.tables);
    S.htab = (uint16_t*)(sbase + lay.htab);
    S.coopCmd = nullptr;
    S.coopStg = nullptr;
    S.job = nullptr;
    uint8_t* inter = sbase + lay.bytes;
    const uint32_t capN = a.capN;
    PhaseProf P;
    P.init(a.prof);
    while (true) {
        uint32_t u = 0;
        if (lane == 0) u = atomicAdd(a.queue, 1u);
        u = __builtin_amdgcn_readfirstlane(u);
        if (u >= a.nchunks) break;
        const size_t c = a.list ? a.list[u] : u;
        const uint32_t n = a.sampleCounts[c];
        int16_t* out = a.samples + a.sampleOffsets[c];
        DecUnit d[kStreams];
        uint64_t total = 0;
        // the claims pass (a.interBytes): any sample count, the frames in an intermediate sized from
        // the listed chunks' claims; a chunk claiming more than it is the claims pass's ALLOC
        const bool claims = a.interBytes != 0;
        int st = (n > capN && !claims) ? PGN_ERR_UNSUPPORTED  // the large-chunk pass takes it
                                       : __builtin_amdgcn_readfirstlane(parse_frames<nf>(
                                             a.in, a.inOffsets[c], a.inSizes[c], d, &total,
                                             claims ? (size_t)a.interBytes : inter_cap(capN)));
        if (claims && st == PGN_ERR_UNSUPPORTED) st = PGN_ERR_ALLOC;
        if (Codec == kCodecC5 && st == PGN_OK && !claims) {  // C5: the staged path's per-stream bound
            uint64_t cs64[kStreams];
            bool over = false;
#pragma unroll
            for (int s = 0; s < nf; s++) {
                cs64[s] = d[s].cs;
                over = over || d[s].cs > capN;
            }
            if (over) st = __builtin_amdgcn_readfirstlane(over_claim_status(a.in, d, cs64, nf));
        }
        if (st == PGN_OK) {
#pragma unroll
            for (int s = 0; s < nf; s++) {  // in blob order (C5.hpp:588-667)
                if (st == PGN_OK) {
                    // VBZ's intermediate carries svb16's 16 padding bytes (signal_compression.cpp:112-118);
                    // the pgnano variants decompress into exactly the content size
                    const size_t cap = Codec == kCodecVbz ? (size_t)d[s].cs + kVbzPadding : (size_t)d[s].cs;
                    const long r = zstd_decompress_wave(a.in + d[s].src, d[s].len, inter + d[s].interOff, cap, S, P);
                    wave_sync();
                    if (r < 0) st = PGN_ERR_ZSTD_DECOMPRESS;
                    d[s].dres = (int32_t)r;
                }
            }
        }
        if (st == PGN_OK) {
            MergeOut mo{0, 0};
            uint64_t want = total;  // the pgnano svb16 decoders need no padding: consume everything
            if (Codec == kCodecVbz) {
                // svb16::decode over content + 16 padding bytes, then "consumed + padding == size"
                // (signal_compression.cpp:100-131): keys running into the padding are "Remaining data"
                const uint64_t padded = total + kVbzPadding;
                if (svb_key_length(n) > total) {
                    mo.bad = svb_key_length(n) <= padded ? 2 : 1;
                } else {
                    mo = vbz_merge_chunk(inter, padded, out, n);
                }
            } else if (Codec == kCodecC1) {
                mo = vbz_merge_chunk(inter, total, out, n);
            } else if (Codec == kCodecVbz0) {
                mo = vbz0_merge_chunk(inter, total, out, n);
            } else if (Codec == kCodecC2 || Codec == kCodecC3) {
                mo = c23_merge_chunk<Codec == kCodecC3>(inter, total, (uint64_t)d[1].dres,
                                                        Codec == kCodecC3 ? (uint64_t)d[2].dres : 0ull, out, n);
            } else {
                mo = c5_merge_chunk<Codec == kCodecC4>(inter, total, (uint64_t)d[1].dres, (uint64_t)d[2].dres,
                                                       (uint64_t)d[3].dres, out, n);
            }
            if (mo.bad == 2) st = PGN_ERR_REMAINING;
            else if (mo.bad) st = PGN_ERR_CORRUPT;
            else if (mo.consumed != want) st = PGN_ERR_REMAINING;
        }
        P.mark(6);
        if (lane == 0) a.status[c] = st;
        wave_sync();
    }
    P.flush();
}

// ---------------------------------------------------------------------------------------------
// Synthetic reads (the checker's pgno_synth_read, oracle/pgn_oracle.c), 64 samples per thread
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t synth_draw(uint64_t rb, uint64_t i, unsigned c)
{
    return mix64(rb + (8ull * i + c + 1ull) * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ int32_t gauss12(uint64_t a, uint64_t b, uint64_t c)
{
    int32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
        s += (int32_t)((a >> (16 * k)) & 0xFFFF) + (int32_t)((b >> (16 * k)) & 0xFFFF) + (int32_t)((c >> (16 * k)) & 0xFFFF);
    return s - 393216;
}

struct SynthArgs {
    size_t nreads;
    uint64_t seed, firstRead, readStride;
    int16_t* samples;
    const uint64_t* offsets;
    const uint32_t* counts;
    uint32_t pq;
    int32_t mean, lsd, nsd;
};

__global__ void synth_kernel(SynthArgs a, uint64_t totalTasks, const uint64_t* taskStart)
{
    // task = (read, 64-sample block); taskStart[r] = first task of read r (prefix sum)
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < totalTasks; t += (uint64_t)gridDim.x * blockDim.x) {
        // binary search the read of task t
        size_t lo = 0, hi = a.nreads;
        while (hi - lo > 1) {
            size_t mid = (lo + hi) / 2;
            if (taskStart[mid] <= t) lo = mid; else hi = mid;
        }
        const size_t r = lo;
        const uint32_t n = a.counts[r];
        const uint32_t i0 = (uint32_t)(t - taskStart[r]) * 64u;
        const uint64_t rid = a.firstRead + r * a.readStride;
        const uint64_t rb = mix64((a.seed << 32) ^ (rid * 0x9E3779B97F4A7C15ull) ^ 0x5851F42D4C957F2Dull);
        // level in force at i0: last switch point <= i0
        uint32_t j = i0;
        while (j > 0 && (uint32_t)(synth_draw(rb, j, 3) >> 48) >= a.pq) j--;
        int32_t level = a.mean + (int32_t)(((int64_t)gauss12(synth_draw(rb, j, 4), synth_draw(rb, j, 5), synth_draw(rb, j, 6)) * a.lsd) >> 16);
        int16_t* out = a.samples + a.offsets[r];
        const uint32_t iend = (i0 + 64 < n) ? i0 + 64 : n;
        for (uint32_t i = i0; i < iend; i++) {
            if (i > i0 && (uint32_t)(synth_draw(rb, i, 3) >> 48) < a.pq)
                level = a.mean + (int32_t)(((int64_t)gauss12(synth_draw(rb, i, 4), synth_draw(rb, i, 5), synth_draw(rb, i, 6)) * a.lsd) >> 16);
            int32_t g = gauss12(synth_draw(rb, i, 0), synth_draw(rb, i, 1), synth_draw(rb, i, 2));
            int32_t v = level + (int32_t)(((int64_t)g * a.nsd) >> 16);
            v = v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
            out[i] = (int16_t)v;
        }
    }
}

__global__ void synth_tasks_kernel(const uint32_t* counts, size_t nreads, uint64_t* taskCount)
{
    for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < nreads; r += (size_t)gridDim.x * blockDim.x)
        taskCount[r] = (counts[r] + 63u) / 64u;
}

// The chunks above kPassSamples of a batch (their indices, in any order), their count and the
// largest sample count among them, and the largest of all: hdr = {count, max large, -, max all},
// zeroed by the caller.
__global__ void large_scan_kernel(const uint32_t* counts, size_t n, uint32_t* list, uint32_t* hdr)
{
    uint32_t mx = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = counts[i];
        mx = v > mx ? v : mx;
        if (v > kPassSamples) {
            list[atomicAdd(hdr, 1u)] = (uint32_t)i;
            atomicMax(hdr + 1, v);
        }
    }
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(hdr + 3, mx);
}

}  // namespace pgn

// =============================================================================================
// Host side: contexts, scratch, launches (C ABI)
// =============================================================================================
using namespace pgn;

// ---- concurrent per-chunk host calls ------------------------------------------------------------
// The reference's readers call the plugin surface from several threads at once (the pod5 async
// signal loader's workers, async_signal_loader.cpp:174-208 -> signal_table_reader.cpp:135-139).  Calls
// on one context that arrive while another is on the device are combined into one small batch
// (flat combining): each call reserves room in the open arena (pinned host memory with a device
// mirror), copies its input there itself, and the first caller that finds the device free runs the
// whole arena as one batch -- one upload, the small-batch kernels for up to kPcMaxReqs chunks, one
// wait -- while later callers fill the other arena.  Each caller copies its own result out.
constexpr int kPcMaxReqs = 64;                    // the small-batch kernels' batch limit
constexpr size_t kPcHdr = 16384;                  // per-request arrays (<= 136 B per request)
constexpr size_t kPcInCap = (size_t)32 << 20;     // input bytes of one arena
constexpr size_t kPcOutCap = (size_t)32 << 20;    // output bytes of one arena
struct PcReq {
    int dir;             // 0 encode, 1 decode
    int codec;
    const void* in;      // samples (encode) or blob (decode), caller's host memory
    size_t inBytes;
    uint32_t n;          // samples
    void* dst;           // encode: blob destination; decode: samples
    size_t cap;          // encode: the destination's capacity
    size_t outBytes;     // room reserved for the result
    size_t inOff, outOff;
    int rc;
    uint64_t outSize;    // encode: blob size (or the required size on PGN_ERR_DST_TOO_SMALL)
    bool done;
};
struct PcArena {
    uint8_t* h = nullptr;     // pinned: [arrays | inputs | outputs]
    uint8_t* hDev = nullptr;  // the device's address of h (the kernels write results there)
    uint8_t* d = nullptr;     // device mirror of [arrays | inputs]
    size_t inUsed = 0, outUsed = 0;
    PcReq* reqs[kPcMaxReqs] = {};
    int nreq = 0, unstaged = 0, readers = 0;
    int state = 0;            // 0 idle / open, 1 on the device, 2 results being copied out
};

struct pgn_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int numCUs = 0;
    size_t encSlotsMax = 0, decSlotsMax = 0;
    // pipeline per direction: the fused per-chunk kernel, or the three-kernel sub-batch pipeline
    // ("staged"); PGN_ENC_PIPELINE / PGN_DEC_PIPELINE = fused | staged override the measured defaults
    bool encStaged = false, decStaged = true;
    // small batches (the per-chunk plugin calls: one chunk) encode on the staged pipeline, whose five
    // stream waves run in parallel: 0.48 ms per 100,000-sample chunk against 0.75 ms for one fused
    // wave; at or below this many chunks (PGN_ENC_STAGED_BELOW; default the CU count) unless
    // PGN_ENC_PIPELINE forces a pipeline
    bool encForced = false;
    size_t encStagedBelow = 0;
    size_t encFusedSlotsMax = 0, decFusedSlotsMax = 0;
    size_t subBatch = 8192;  // chunks per pipeline pass (PGN_SUBBATCH, staged pipeline)
    // C5 decode batches of at least deferMin chunks defer their four-stream Huffman sections to
    // dec_huf_kernel (pgn_hufjob.h), in passes of up to deferG chunks: a lane-per-stream decoder
    // needs thousands of frames in flight (PGN_DEFER_MIN_CHUNKS / PGN_DEFER_G tune both; the output
    // is the same either way)
    size_t deferMin = 12288, deferG = 12500;
    // the last pass of a deferred call decodes its Huffman sections in place (dec_zstd_kernel's 16-
    // lanes-per-stream decoder): this many chunks (PGN_DEFER_TAIL_PLAIN; 0 = every pass deferred).
    // A deferred pass ends with one lane's ~16,000-symbol chain per M stream, which nothing overlaps
    // once the frame decode of the last pass is done (the decode's drain)
    size_t deferTailPlain = 0;
    size_t deferHead = 0;      // PGN_DEFER_HEAD: chunks of a short first deferred pass (0 = balanced passes)
    bool hufPrioLast = false;  // PGN_HUF_PRIO_LAST=1: the last deferred pass's dec_huf waves at raised priority
    bool lastOnCaller = false;  // PGN_LAST_ON_CALLER=1: the last deferred pass's sections and merge on the caller's stream
    size_t hufWideLast = 0;    // PGN_HUF_WIDE_LAST: the last this many deferred passes decode their sections with dec_huf_wide_kernel
    bool lastDeferred = false;  // the last staged C5 decode deferred its Huffman sections (pgn_ctx_kernels)
    // encode: per-slot scratch of the zstd kernel, per-chunk streams/frames of one sub-batch
    uint8_t* encScratch = nullptr;
    size_t encSlots = 0;
    uint32_t* epochs = nullptr;
    uint8_t* encChunks = nullptr;  // per buffer: G * (kChunkStreamBytes + kChunkFrameBytes) + sizes + fsizes
    size_t encG = 0;               // chunk capacity of all buffers together
    // decode
    uint8_t* decScratch = nullptr;
    size_t decSlots = 0;
    uint8_t* decChunks = nullptr;  // per buffer: G * interStride + units (+ Huffman jobs)
    size_t decBytes = 0;
    DecUnit* lastUnits = nullptr;  // decode records of the last pass (diagnostics)
    size_t lastG = 0;              // ... for this many chunks
    uint32_t* queues = nullptr;    // a ring of work counters, zeroed when it wraps (one per sub-batch pass)
    size_t qNext = 0;              // next unused counter of the ring
    uint32_t* qCur = nullptr;      // the current call's counters
    uint64_t* lookback = nullptr;  // dec_merge_lb_kernel's published words (kMergeWgMaxChunks chunks)
    uint64_t lbEpoch = 0;          // the tag of the last call that used them
    size_t nQueues = 0;
    // host-call staging: a device buffer and its pinned host mirror (same layout), so a per-chunk
    // call is one upload, the launches and one download
    uint8_t* stage = nullptr;
    uint8_t* hstage = nullptr;
    uint8_t* hstageDev = nullptr;  // the device's address of hstage (kernels write the call's outputs there)
    size_t stageBytes = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // two-stream pipeline over sub-batches (launch_encode / launch_decode): the side stream runs the
    // split (encode) or the merge (decode) of one sub-batch while the caller's stream runs the zstd
    // kernel of the neighbouring one; two per-chunk buffers alternate between sub-batches
    hipStream_t side = nullptr;
    hipEvent_t evFork = nullptr, evJoin = nullptr, evStage[2] = {nullptr, nullptr}, evFree[2] = {nullptr, nullptr};
    // deferred-Huffman decode passes: the merges on a third stream, so the merge of pass p (VALU-bound)
    // can share the CUs with the Huffman sections of pass p + 1 (latency-bound)
    hipStream_t mergeS = nullptr;
    hipEvent_t evHuf[2] = {nullptr, nullptr};
    // decode passes: buffers in rotation (PGN_DEC_BUFS, 2..kMaxDecBufs) with their stage / sections /
    // free events, and the streams the deferred sections alternate over (PGN_HUF_STREAMS: 1 or 2 with
    // the merges on mergeS; 3 = sections and merge of pass p both on side stream p % 3 of side, side2,
    // mergeS).  Measured (tools/gpu_env_sweep.sh, 100,000 chunks): 2 buffers / 1 stream / passes of
    // 20,000: decode 23.1 ms; 4 / 2 / 12,500: 22.7 ms; 4 / 3 / 12,500: 22.3-22.6 ms against 22.8-23.1
    // in interleaved A/B (profiles/r05_decode_pipeline_sweep.log)
    size_t decBufs = 4, hufStreams = 3;
    hipStream_t side2 = nullptr;
    hipEvent_t evDStage[kMaxDecBufs] = {}, evDHuf[kMaxDecBufs] = {}, evDFree[kMaxDecBufs] = {};
    uint64_t* prof = nullptr;  // kProfWords: phase cycles and counters (encode, decode, dec_huf) when PGN_PHASE_PROFILE=1
    bool encTimed = false, decTimed = false;
    // Stream ordering of the context's shared state (work counters, slot scratch, per-chunk buffers):
    // every launch sequence records evLast on its stream at the end, and the next one, on whatever
    // stream, waits for it before touching that state.  Calls on one context therefore run in call
    // order on the device even when callers pass different streams.
    hipEvent_t evLast = nullptr;
    bool haveLast = false;
    // Large-chunk pass (chunks above kPassSamples, launch_large): the chunk list, its header
    // {count, largest} on the device and in pinned memory, read on a stream of its own while the
    // batched pass runs; slot scratch spaced for the largest chunk, and its own table epochs and
    // work counter.
    uint32_t* largeList = nullptr;
    uint32_t* claimList = nullptr;     // the claims pass's chunks (claim_scan_kernel, or from the host)
    size_t largeListCap = 0;
    uint32_t* largeHdr = nullptr;      // [0..1] header, [2] the large pass's work counter, [3] largest chunk,
                                       // [4..5] the claims pass's count and largest sum (KiB)
    uint32_t* largeHdrHost = nullptr;
    hipStream_t scanStream = nullptr;
    hipEvent_t evScanFork = nullptr, evScan = nullptr;
    // the encode and the decode of the large pass keep separate slot scratch: the encoder's hash
    // tables persist across calls (epoch tags), so a decode must never write over them
    uint8_t* largeScratch = nullptr;
    size_t largeScratchBytes = 0;
    uint32_t* largeEpochs = nullptr;
    size_t largeEpochSlots = 0;
    uint8_t* largeDecScratch = nullptr;
    size_t largeDecScratchBytes = 0;
    std::mutex mu;
    // combined per-chunk host calls (PcArena): pcOpen = the arena new calls join (-1: none idle)
    std::mutex pcMu;
    std::condition_variable pcCv;
    PcArena pcA[2];
    int pcOpen = 0;
    bool pcBusy = false;
    int pcReady = 0;  // 0 not yet allocated, 1 ready, -1 allocation failed (calls run one by one)
};

static thread_local char g_err[512];

static int hip_fail(hipError_t e, const char* what)
{
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return PGN_ERR_HIP;
}
#define HIPCHK(x)                                   \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #x); \
    } while (0)

extern "C" {

const char* pgn_status_string(int s)
{
    switch (s) {
    case PGN_OK: return "OK";
    case PGN_ERR_DST_TOO_SMALL: return "Not enough space in destination buffer";
    case PGN_ERR_NOT_ZSTD: return "Input data not compressed by zstd";
    case PGN_ERR_ZSTD_DECOMPRESS: return "Input data failed to decompress using zstd";
    case PGN_ERR_REMAINING: return "Remaining data at end of signal buffer";
    case PGN_ERR_ZSTD_COMPRESS: return "Failed to compress data";
    case PGN_ERR_CORRUPT: return "Corrupt compressed signal (stream read past its end)";
    case PGN_ERR_ALLOC: return "Out of memory: the frames' content sizes sum to more than 2^40 bytes";
    case PGN_ERR_UNSUPPORTED: return "Chunk larger than PGN_MAX_CHUNK_SAMPLES, or frames expanding beyond the decoder's buffer";
    case PGN_ERR_INVALID_ARG: return "Invalid argument";
    case PGN_ERR_HIP: return "HIP runtime error";
    case PGN_ERR_NO_DEVICE: return "No HIP device";
    case PGN_ERR_IO: return "File I/O failure";
    default: return "Unknown status";
    }
}

const char* pgn_last_error(void) { return g_err; }

size_t pgn_compressed_signal_max_size(size_t n)
{
    size_t s = n * 2 + 10 + 16;
    return s > 1024 ? s : 1024;
}

int pgn_ctx_create(int device, pgn_ctx** out)
{
    if (!out) return PGN_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PGN_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return PGN_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(device));
    pgn_ctx* c = new pgn_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    c->numCUs = prop.multiProcessorCount;
    int encPerCU = 0, decPerCU = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&encPerCU, enc_zstd_kernel, 64, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&decPerCU, dec_zstd_kernel, 64, 0));
    int fe = 0, fd = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&fe, enc_chunk_kernel<kCodecC5>, 64, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&fd, dec_chunk_kernel<kCodecC5>, 64, 0));
    if (fe < 1) fe = 1;
    if (fd < 1) fd = 1;
    if (const char* v = getenv("PGN_ENC_WG_PER_CU")) { const int x = atoi(v); if (x > 0 && x < fe) fe = x; }
    if (const char* v = getenv("PGN_DEC_WG_PER_CU")) { const int x = atoi(v); if (x > 0 && x < fd) fd = x; }
    c->encFusedSlotsMax = (size_t)c->numCUs * (size_t)(fe > 32 ? 32 : fe);
    c->decFusedSlotsMax = (size_t)c->numCUs * (size_t)(fd > 32 ? 32 : fd);
    if (encPerCU < 1) encPerCU = 1;
    if (decPerCU < 1) decPerCU = 1;
    // resident zstd workgroups per CU (tuning knobs PGN_ENC_WG_PER_CU / PGN_DEC_WG_PER_CU: fewer
    // leave room for the side stream's split / merge kernels)
    if (const char* v = getenv("PGN_ENC_WG_PER_CU")) { const int x = atoi(v); if (x > 0 && x < encPerCU) encPerCU = x; }
    if (const char* v = getenv("PGN_DEC_WG_PER_CU")) { const int x = atoi(v); if (x > 0 && x < decPerCU) decPerCU = x; }
    c->encSlotsMax = (size_t)c->numCUs * (size_t)(encPerCU > 32 ? 32 : encPerCU);
    c->decSlotsMax = (size_t)c->numCUs * (size_t)(decPerCU > 32 ? 32 : decPerCU);
    c->encStagedBelow = (size_t)c->numCUs;
    if (const char* v = getenv("PGN_ENC_STAGED_BELOW")) c->encStagedBelow = (size_t)atol(v);
    if (const char* pp = getenv("PGN_ENC_PIPELINE")) {
        c->encStaged = strcmp(pp, "staged") == 0;
        c->encForced = true;
    }
    if (const char* pp = getenv("PGN_DEC_PIPELINE")) c->decStaged = strcmp(pp, "staged") == 0;
    if (const char* sb = getenv("PGN_SUBBATCH")) {
        long v = atol(sb);
        if (v > 0) c->subBatch = (size_t)v;
    }
    if (const char* v = getenv("PGN_DEFER_MIN_CHUNKS")) { const long x = atol(v); if (x > 0) c->deferMin = (size_t)x; }
    if (const char* v = getenv("PGN_DEFER_G")) { const long x = atol(v); if (x > 0) c->deferG = (size_t)x; }
    if (const char* v = getenv("PGN_DEFER_HEAD")) { const long x = atol(v); if (x >= 0) c->deferHead = (size_t)x; }
    if (const char* v = getenv("PGN_LAST_ON_CALLER")) c->lastOnCaller = v[0] == '1';
    if (const char* v = getenv("PGN_HUF_WIDE_LAST")) { const long x = atol(v); if (x >= 0) c->hufWideLast = (size_t)x; }
    if (const char* v = getenv("PGN_HUF_PRIO_LAST")) c->hufPrioLast = v[0] == '1';
    if (const char* v = getenv("PGN_DEFER_TAIL_PLAIN")) { const long x = atol(v); if (x >= 0) c->deferTailPlain = (size_t)x; }
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    const char* pe = getenv("PGN_PHASE_PROFILE");
    if (pe && pe[0] == '1') {
        // [encode phases][decode phases][encode counters][decode counters]
        HIPCHK(hipMalloc(&c->prof, kProfWords * sizeof(uint64_t)));
        HIPCHK(hipMemset(c->prof, 0, kProfWords * sizeof(uint64_t)));
        HIPCHK(hipDeviceSynchronize());
    }
    for (int i = 0; i < 4; i++) HIPCHK(hipEventCreate(&c->ev[i]));
    HIPCHK(hipEventCreateWithFlags(&c->evLast, hipEventDisableTiming));
    HIPCHK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->mergeS, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking));
    for (int i = 0; i < kMaxDecBufs; i++) {
        HIPCHK(hipEventCreateWithFlags(&c->evDStage[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->evDHuf[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->evDFree[i], hipEventDisableTiming));
    }
    if (const char* v = getenv("PGN_DEC_BUFS")) {
        const long x = atol(v);
        if (x >= 2 && x <= kMaxDecBufs) c->decBufs = (size_t)x;
    }
    if (const char* v = getenv("PGN_HUF_STREAMS")) {
        const long x = atol(v);
        c->hufStreams = x >= 1 && x <= 3 ? (size_t)x : c->hufStreams;
    }
    HIPCHK(hipStreamCreateWithFlags(&c->scanStream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c->evScanFork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->evScan, hipEventDisableTiming));
    HIPCHK(hipMalloc(&c->largeHdr, 8 * sizeof(uint32_t)));
    HIPCHK(hipHostMalloc((void**)&c->largeHdrHost, 8 * sizeof(uint32_t), hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&c->evFork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->evJoin, hipEventDisableTiming));
    for (int i = 0; i < 2; i++) {
        HIPCHK(hipEventCreateWithFlags(&c->evStage[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->evFree[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->evHuf[i], hipEventDisableTiming));
    }
    // the predefined sequence FSE tables of the decoder (one wave, once per context)
    hipLaunchKernelGGL(seq_default_tables_kernel, dim3(1), dim3(64), 0, c->stream);
    HIPCHK(hipGetLastError());
    // and the encoder's
    hipLaunchKernelGGL(seq_default_ctables_kernel, dim3(1), dim3(64), 0, c->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    *out = c;
    return PGN_OK;
}

int pgn_ctx_destroy(pgn_ctx* c)
{
    if (!c) return PGN_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->encScratch);
    (void)hipFree(c->epochs);
    (void)hipFree(c->decScratch);
    (void)hipFree(c->encChunks);
    (void)hipFree(c->decChunks);
    (void)hipFree(c->queues);
    (void)hipFree(c->lookback);
    (void)hipFree(c->stage);
    if (c->hstage) (void)hipHostFree(c->hstage);
    (void)hipFree(c->prof);
    for (PcArena& A : c->pcA) {
        if (A.h) (void)hipHostFree(A.h);
        (void)hipFree(A.d);
    }
    if (c->scanStream) (void)hipStreamSynchronize(c->scanStream);
    (void)hipFree(c->largeList);
    (void)hipFree(c->claimList);
    (void)hipFree(c->largeHdr);
    (void)hipFree(c->largeScratch);
    (void)hipFree(c->largeEpochs);
    (void)hipFree(c->largeDecScratch);
    if (c->largeHdrHost) (void)hipHostFree(c->largeHdrHost);
    for (hipEvent_t e : {c->evScanFork, c->evScan})
        if (e) (void)hipEventDestroy(e);
    if (c->scanStream) (void)hipStreamDestroy(c->scanStream);
    for (int i = 0; i < 4; i++) if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->mergeS) (void)hipStreamSynchronize(c->mergeS);
    if (c->side2) (void)hipStreamSynchronize(c->side2);
    for (int i = 0; i < kMaxDecBufs; i++)
        for (hipEvent_t e : {c->evDStage[i], c->evDHuf[i], c->evDFree[i]})
            if (e) (void)hipEventDestroy(e);
    if (c->evLast) (void)hipEventSynchronize(c->evLast);
    for (hipEvent_t e : {c->evFork, c->evJoin, c->evStage[0], c->evStage[1], c->evFree[0], c->evFree[1], c->evLast, c->evHuf[0],
                         c->evHuf[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->mergeS) (void)hipStreamDestroy(c->mergeS);
    if (c->side2) (void)hipStreamDestroy(c->side2);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return PGN_OK;
}

void* pgn_ctx_stream(pgn_ctx* c) { return c ? (void*)c->stream : nullptr; }

// The last launch sequence on any stream (evLast) has finished with the context's buffers.
static void wait_last_host(pgn_ctx* c)
{
    if (c->haveLast) (void)hipEventSynchronize(c->evLast);
    (void)hipStreamSynchronize(c->stream);
}

static int ensure_enc(pgn_ctx* c, size_t slots, size_t G)
{
    if (slots > c->encSlots) {
        wait_last_host(c);
        (void)hipFree(c->encScratch);
        (void)hipFree(c->epochs);
        c->encScratch = nullptr;
        c->epochs = nullptr;
        const size_t sb = enc_slot_bytes();
        HIPCHK(hipMalloc(&c->encScratch, sb * slots));
        HIPCHK(hipMalloc(&c->epochs, 4 * slots));
        // tag 0 never matches: a zeroed table is an empty table for every epoch >= 1.  The context
        // stream is non-blocking, so zero on it and wait before any launch (on any stream) uses it.
        HIPCHK(hipMemsetAsync(c->epochs, 0, 4 * slots, c->stream));
        HIPCHK(hipMemsetAsync(c->encScratch, 0, sb * slots, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->encSlots = slots;
    }
    if (G > c->encG) {  // G = chunk capacity over all buffers
        wait_last_host(c);
        (void)hipDeviceSynchronize();
        (void)hipFree(c->encChunks);
        c->encChunks = nullptr;
        HIPCHK(hipMalloc(&c->encChunks, G * (kChunkStreamBytes + kChunkFrameBytes + 2 * 4 * kStreams)));
        c->encG = G;
    }
    return PGN_OK;
}

static int ensure_dec(pgn_ctx* c, size_t slots, size_t bytes)
{
    if (slots > c->decSlots) {
        wait_last_host(c);
        (void)hipFree(c->decScratch);
        c->decScratch = nullptr;
        HIPCHK(hipMalloc(&c->decScratch, dec_slot_bytes() * slots));
        c->decSlots = slots;
    }
    if (bytes > c->decBytes) {  // the per-chunk buffers of all passes in flight
        wait_last_host(c);
        (void)hipDeviceSynchronize();
        (void)hipFree(c->decChunks);
        c->decChunks = nullptr;
        HIPCHK(hipMalloc(&c->decChunks, bytes));
        c->decBytes = bytes;
    }
    return PGN_OK;
}

// The look-back words of the small-batch range split / merge and this call's tag.  Launch sequences
// on a context are ordered (evLast), so one array serves every call; it is cleared when the 16-bit
// tags wrap.
static int take_lookback(pgn_ctx* c, hipStream_t s, uint64_t*& words, uint64_t& epoch)
{
    const size_t bytes = sizeof(uint64_t) * 3 * 32 * 64;  // 3 words x 32 ranges x 64 chunks
    if (!c->lookback) {
        HIPCHK(hipMalloc(&c->lookback, bytes));
        HIPCHK(hipMemsetAsync(c->lookback, 0, bytes, s));
    }
    if (++c->lbEpoch > 0xFFFFu) {
        HIPCHK(hipMemsetAsync(c->lookback, 0, bytes, s));
        c->lbEpoch = 1;
    }
    words = c->lookback;
    epoch = c->lbEpoch;
    return PGN_OK;
}

// n fresh zeroed work counters for this call (c->qCur).  The counters come from a ring that is zeroed
// only when it wraps: a per-call memset was a fill kernel plus a launch gap in front of every
// per-chunk call.  Launch sequences on a context are ordered (evLast), so the wrap's memset runs
// after every earlier user of the ring.
static int ensure_queues(pgn_ctx* c, size_t n, hipStream_t s)
{
    constexpr size_t kRing = 1 << 14;
    if (!c->queues || n > c->nQueues) {
        wait_last_host(c);
        (void)hipStreamSynchronize(s);
        (void)hipFree(c->queues);
        c->queues = nullptr;
        const size_t m = n < kRing ? kRing : n;
        HIPCHK(hipMalloc(&c->queues, 4 * m));
        HIPCHK(hipMemsetAsync(c->queues, 0, 4 * m, s));
        c->nQueues = m;
        c->qNext = 0;
    }
    if (c->qNext + n > c->nQueues) {
        HIPCHK(hipMemsetAsync(c->queues, 0, 4 * c->nQueues, s));
        c->qNext = 0;
    }
    c->qCur = c->queues + c->qNext;
    c->qNext += n;
    return PGN_OK;
}

static int launch_enc_chunks(int codec, const EncArgs& a, size_t slots, hipStream_t s);
static int launch_dec_chunks(int codec, const DecArgs& a, size_t slots, hipStream_t s);

static int launch_encode_fused(pgn_ctx* c, int codec, size_t nchunks, const int16_t* d_samples,
                               const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out,
                               const uint64_t* d_out_offsets, const uint64_t* d_out_caps, uint64_t* d_out_sizes,
                               int32_t* d_status, uint64_t* d_stats, hipStream_t s)
{
    const size_t slots = nchunks < c->encFusedSlotsMax ? nchunks : c->encFusedSlotsMax;
    int rc = ensure_enc(c, slots, 0);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev[0], s));
    rc = ensure_queues(c, 1, s);
    if (rc) return rc;
    EncArgs a{};
    a.nchunks = nchunks;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.out = d_out;
    a.outOffsets = d_out_offsets;
    a.outCaps = d_out_caps;
    a.outSizes = d_out_sizes;
    a.status = d_status;
    a.stats = d_stats;
    a.slotScratch = c->encScratch;
    a.slotBytes = enc_slot_bytes();
    a.epochs = c->epochs;
    a.prof = c->prof;
    a.queue = c->qCur;
    a.capN = kPassSamples;
    a.list = nullptr;
    return launch_enc_chunks(codec, a, slots, s);
}

static int launch_enc_chunks(int codec, const EncArgs& a, size_t slots, hipStream_t s)
{
    switch (codec) {
    case kCodecC5: hipLaunchKernelGGL(enc_chunk_kernel<kCodecC5>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecVbz: hipLaunchKernelGGL(enc_chunk_kernel<kCodecVbz>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC4: hipLaunchKernelGGL(enc_chunk_kernel<kCodecC4>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC1: hipLaunchKernelGGL(enc_chunk_kernel<kCodecC1>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC2: hipLaunchKernelGGL(enc_chunk_kernel<kCodecC2>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC3: hipLaunchKernelGGL(enc_chunk_kernel<kCodecC3>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecVbz0: hipLaunchKernelGGL(enc_chunk_kernel<kCodecVbz0>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    default: return PGN_ERR_INVALID_ARG;
    }
    HIPCHK(hipGetLastError());
    return PGN_OK;
}

static int launch_decode_fused(pgn_ctx* c, int codec, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                               const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                               const uint32_t* d_sample_counts, int32_t* d_status, hipStream_t s)
{
    const size_t slots = nchunks < c->decFusedSlotsMax ? nchunks : c->decFusedSlotsMax;
    int rc = ensure_dec(c, slots, 0);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev[2], s));
    rc = ensure_queues(c, 1, s);
    if (rc) return rc;
    DecArgs a{};
    a.nchunks = nchunks;
    a.in = d_in;
    a.inOffsets = d_in_offsets;
    a.inSizes = d_in_sizes;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.status = d_status;
    a.slotScratch = c->decScratch;
    a.slotBytes = dec_slot_bytes();
    a.prof = c->prof ? c->prof + kPhases : nullptr;
    a.queue = c->qCur;
    a.capN = kPassSamples;
    a.list = nullptr;
    c->lastUnits = nullptr;
    return launch_dec_chunks(codec, a, slots, s);
}

static int launch_dec_chunks(int codec, const DecArgs& a, size_t slots, hipStream_t s)
{
    switch (codec) {
    case kCodecC5: hipLaunchKernelGGL(dec_chunk_kernel<kCodecC5>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecVbz: hipLaunchKernelGGL(dec_chunk_kernel<kCodecVbz>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC4: hipLaunchKernelGGL(dec_chunk_kernel<kCodecC4>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC1: hipLaunchKernelGGL(dec_chunk_kernel<kCodecC1>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC2: hipLaunchKernelGGL(dec_chunk_kernel<kCodecC2>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecC3: hipLaunchKernelGGL(dec_chunk_kernel<kCodecC3>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    case kCodecVbz0: hipLaunchKernelGGL(dec_chunk_kernel<kCodecVbz0>, dim3((unsigned)slots), dim3(64), 0, s, a); break;
    default: return PGN_ERR_INVALID_ARG;
    }
    HIPCHK(hipGetLastError());
    return PGN_OK;
}

static int launch_encode_impl(pgn_ctx* c, int codec, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                         const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                         void* stream)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const bool staged = c->encStaged || (!c->encForced && nchunks <= c->encStagedBelow);
    if (!staged || (codec != kCodecC5 && codec != kCodecVbz))  // the other variants are fused only
        return launch_encode_fused(c, codec, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                                   d_out_caps, d_out_sizes, d_status, d_stats, s);
    const size_t G = nchunks < c->subBatch ? nchunks : c->subBatch;
    const size_t passes = (nchunks + G - 1) / G;
    const uint32_t nu = codec == kCodecVbz ? 1u : (uint32_t)kStreams;
    const size_t slots = nu * G < c->encSlotsMax ? nu * G : c->encSlotsMax;
    const size_t nbuf = passes > 1 ? 2 : 1;
    int rc = ensure_enc(c, slots, nbuf * G);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev[0], s));
    rc = ensure_queues(c, passes, s);
    if (rc) return rc;
    // the split of pass p + 1 runs on the side stream beside pass p's zstd kernel; a single pass
    // stays on the caller's stream (no fork, no cross-stream events)
    const hipStream_t sideS = passes > 1 ? c->side : s;
    if (passes > 1) {
        HIPCHK(hipEventRecord(c->evFork, s));
        HIPCHK(hipStreamWaitEvent(c->side, c->evFork, 0));
    }
    const size_t bufBytes = G * (kChunkStreamBytes + kChunkFrameBytes + 2 * 4 * kStreams);
    EncArgs a;
    a.nchunks = nchunks;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.out = d_out;
    a.outOffsets = d_out_offsets;
    a.outCaps = d_out_caps;
    a.outSizes = d_out_sizes;
    a.status = d_status;
    a.stats = d_stats;
    a.slotScratch = c->encScratch;
    a.slotBytes = enc_slot_bytes();
    a.epochs = c->epochs;
    a.prof = c->prof;
    a.G = G;
    a.nu = nu;
    a.capN = kPassSamples;
    a.list = nullptr;
    a.lookback = nullptr;
    a.epoch = 0;
    if (passes == 1 && G <= kSplitWgMaxChunks && codec != kCodecVbz) {  // the look-back range split (one epoch per pass)
        rc = take_lookback(c, s, a.lookback, a.epoch);
        if (rc) return rc;
    }
    // pass p: split on the side stream into buffer p % 2; zstd + assemble on the caller's stream.
    // The split of pass p+1 overlaps the zstd kernel of pass p; a buffer is split into again only
    // after the assemble kernel of the pass before last has read it.
    for (size_t p = 0; p < passes; p++) {
        const int b = (int)(p & 1);
        uint8_t* buf = c->encChunks + (size_t)b * bufBytes;
        a.streams = buf;
        a.frames = buf + G * kChunkStreamBytes;
        a.sizes = (uint32_t*)(a.frames + G * kChunkFrameBytes);
        a.fsizes = a.sizes + G * kStreams;
        a.base = p * G;
        a.queue = c->qCur + p;
        if (p >= 2) HIPCHK(hipStreamWaitEvent(c->side, c->evFree[b], 0));
        if (codec == kCodecVbz) hipLaunchKernelGGL(vbz_split_kernel, dim3((unsigned)G), dim3(64), 0, sideS, a);
        else if (a.lookback)  // few chunks: kSplitRanges single-wave workgroups per chunk
            hipLaunchKernelGGL(enc_split_lb_kernel, dim3((unsigned)(G * kSplitRanges)), dim3(64), 0, sideS, a);
        else hipLaunchKernelGGL(enc_split_kernel, dim3((unsigned)G), dim3(64), 0, sideS, a);
        if (passes > 1) {
            HIPCHK(hipEventRecord(c->evStage[b], c->side));
            HIPCHK(hipStreamWaitEvent(s, c->evStage[b], 0));
        }
        const bool coop = G <= kSplitWgMaxChunks && (size_t)nu * G <= slots;
        if (coop)  // few chunks: a workgroup per stream (C5: the frames place themselves, enc_place_frame)
            hipLaunchKernelGGL(enc_zstd_coop_kernel, dim3((unsigned)(nu * G)), dim3(64 * kCoopEncWaves), 0, s, a);
        else hipLaunchKernelGGL(enc_zstd_kernel, dim3((unsigned)slots), dim3(64), 0, s, a);
        if (codec == kCodecVbz) hipLaunchKernelGGL(vbz_assemble_kernel, dim3((unsigned)G), dim3(64), 0, s, a);
        else if (!(coop && a.lookback)) hipLaunchKernelGGL(enc_assemble_kernel, dim3((unsigned)G), dim3(64), 0, s, a);
        if (passes > 1) HIPCHK(hipEventRecord(c->evFree[b], s));
    }
    HIPCHK(hipGetLastError());
    return PGN_OK;
}

// capCall: every chunk of the call has at most this many samples (a multiple of 4096, at most
// kPassSamples); the per-chunk intermediates are spaced for it.
static int launch_decode_impl(pgn_ctx* c, int codec, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                         const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, int32_t* d_status, void* stream, uint32_t capCall)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (!c->decStaged || (codec != kCodecC5 && codec != kCodecVbz))
        return launch_decode_fused(c, codec, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                                   d_sample_counts, d_status, s);
    // large C5 batches: deferred Huffman sections (dec_huf_kernel), passes of up to deferG chunks
    // balanced over the batch; otherwise passes of subBatch chunks
    bool defer = codec == kCodecC5 && nchunks >= c->deferMin;
    const size_t stride = chunk_inter_bytes(capCall);
    size_t G = nchunks < c->subBatch ? nchunks : c->subBatch;  // chunks per pass (the buffers' capacity)
    // the passes: chunks [pBase[p], pBase[p] + pCnt[p]); pPlain[p]: a deferred call's in-place tail
    std::vector<size_t> pBase, pCnt;
    std::vector<char> pPlain;
    if (defer) {  // up to deferG chunks per pass, and decBufs passes' buffers within kDecBufferBudget
        // (the budget's bound is at least subBatch chunks; PGN_DEFER_G below that is the tests' way to
        // run several passes on small batches)
        size_t gmax = kDecBufferBudget / (c->decBufs * (stride + kStreams * (sizeof(DecUnit) + kJobBytes)));
        gmax = gmax < c->subBatch ? c->subBatch : gmax;
        gmax = gmax < c->deferG ? gmax : c->deferG;
        // an optional short first pass (PGN_DEFER_HEAD: the sections start sooner), the passes of up to
        // gmax chunks balanced over the rest, and an optional in-place tail pass (PGN_DEFER_TAIL_PLAIN)
        size_t head = c->deferHead, tail = c->deferTailPlain;
        if (!(head > 0 && head <= gmax && nchunks >= 4 * head)) head = 0;
        if (!(tail > 0 && tail <= gmax && nchunks - head >= 2 * tail)) tail = 0;
        if (head) {
            pBase.push_back(0);
            pCnt.push_back(head);
            pPlain.push_back(0);
        }
        const size_t mid = nchunks - head - tail;
        const size_t np = (mid + gmax - 1) / gmax;
        const size_t Gd = (mid + np - 1) / np;
        for (size_t b = head; b < head + mid; b += Gd) {
            pBase.push_back(b);
            pCnt.push_back(head + mid - b < Gd ? head + mid - b : Gd);
            pPlain.push_back(0);
        }
        if (tail) {
            pBase.push_back(nchunks - tail);
            pCnt.push_back(tail);
            pPlain.push_back(1);
        }
        G = 0;
        for (size_t k : pCnt) G = k > G ? k : G;
    } else {
        for (size_t b = 0; b < nchunks; b += G) {
            pBase.push_back(b);
            pCnt.push_back(G);  // the kernels stop at nchunks
            pPlain.push_back(1);
        }
    }
    const size_t passes = pBase.size();
    size_t nDefPasses = 0;  // deferred passes (an in-place tail pass comes last)
    for (size_t p = 0; p < passes; p++) nDefPasses += defer && !pPlain[p] ? 1 : 0;
    const uint32_t nu = codec == kCodecVbz ? 1u : (uint32_t)kStreams;
    const size_t slots = nu * G < c->decSlotsMax ? nu * G : c->decSlotsMax;
    // few chunks: a workgroup per frame (not for the passes of a larger deferred call)
    const bool coop = G <= kCoopMaxChunks && (size_t)nu * G <= slots && !(defer && nchunks > kCoopMaxChunks);
    defer = defer && !coop;  // the cooperative kernel decodes its sections itself
    c->lastDeferred = defer;
    // buffers in rotation: a pass parses into buffer p % nbuf once the merge of pass p - nbuf has read it
    const size_t nbuf = passes > 1 ? (passes < c->decBufs ? passes : c->decBufs) : 1;
    const size_t unitBytes = align_up(G * kStreams * sizeof(DecUnit), 256);
    const size_t bufBytes = G * stride + unitBytes + (defer ? G * kStreams * kJobBytes + kHufJunkBytes : 0);
    int rc = ensure_dec(c, slots, nbuf * bufBytes);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev[2], s));
    rc = ensure_queues(c, passes, s);
    if (rc) return rc;
    // the merge of pass p runs on the side stream beside pass p + 1's zstd kernel; a single pass
    // stays on the caller's stream
#ifdef PGN_SERIAL_DECODE  // diagnostic builds: every decode kernel on the caller's stream (isolated kernel times)
    const hipStream_t sideS = s;
    const bool multi = false;
#else
    const hipStream_t sideS = passes > 1 ? c->side : s;
    const bool multi = passes > 1;
#endif
    // deferred sections over several passes: the sections of pass p on hufS[p % hufStreams], the merges
    // on a third stream behind them
    // 3: the sections and the merge of pass p both on side stream p % 3 (no separate merge stream)
    const hipStream_t hufS[3] = {c->side, c->side2, c->mergeS};
    const size_t hufStreams = c->hufStreams;
    if (passes > 1) {
        HIPCHK(hipEventRecord(c->evFork, s));
        HIPCHK(hipStreamWaitEvent(c->side, c->evFork, 0));
    }
    DecArgs a{};
    a.nchunks = nchunks;
    a.in = d_in;
    a.inOffsets = d_in_offsets;
    a.inSizes = d_in_sizes;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.status = d_status;
    a.slotScratch = c->decScratch;
    a.slotBytes = dec_slot_bytes();
    a.prof = c->prof ? c->prof + kPhases : nullptr;
    a.G = G;
    a.nu = nu;
    a.capN = capCall;
    a.interStride = stride;
    a.list = nullptr;
    a.lookback = nullptr;
    a.epoch = 0;
    if (passes == 1 && G <= kMergeWgMaxChunks && codec != kCodecVbz) {  // the look-back range merge (one epoch per pass)
        const int lrc = take_lookback(c, s, a.lookback, a.epoch);
        if (lrc) return lrc;
    }
    // pass p: parse + zstd on the caller's stream into buffer p % nbuf, the deferred Huffman sections
    // and the merge on the side streams.  Those of pass p overlap the zstd kernel of pass p+1.
    for (size_t p = 0; p < passes; p++) {
        const int b = (int)(p % nbuf);
        uint8_t* buf = c->decChunks + (size_t)b * bufBytes;
        const bool deferP = defer && !pPlain[p];
        a.base = pBase[p];
        a.G = pCnt[p];
        a.inter = buf;
        a.units = (DecUnit*)(buf + G * stride);
        a.jobs = deferP ? buf + G * stride + unitBytes : nullptr;
        // the last deferred pass's sections: nothing after them overlaps their chains
        a.hufPrio = (deferP && c->hufPrioLast && (p + 1 == passes || (p + 2 == passes && pPlain[passes - 1]))) ? 1u : 0u;
        c->lastUnits = a.units;
        c->lastG = a.G;
        a.queue = c->qCur + p;
        if (p >= nbuf) HIPCHK(hipStreamWaitEvent(s, c->evDFree[b], 0));
        a.coopParse = (coop && codec != kCodecVbz) ? 1u : 0u;
        if (codec == kCodecVbz) hipLaunchKernelGGL(vbz_parse_kernel, dim3((unsigned)((G + 63) / 64)), dim3(64), 0, s, a);
        else if (!a.coopParse) hipLaunchKernelGGL(dec_parse_kernel, dim3((unsigned)((G + 63) / 64)), dim3(64), 0, s, a);
        if (coop)
            hipLaunchKernelGGL(dec_zstd_coop_kernel, dim3((unsigned)(nu * G)), dim3(64 * kCoopWaves), 0, s, a);
        else hipLaunchKernelGGL(dec_zstd_kernel, dim3((unsigned)slots), dim3(64), 0, s, a);
        // the stream of this pass's sections (deferred) or merge (otherwise)
        // (the last pass's on the caller's stream, right behind its frame decode: on side stream p % 3
        // they would queue behind pass p - 3's merge, which ends ~1 ms after the frame decode,
        // profiles/r06_decode_timeline_a.txt)
        const bool lastOnCaller = defer && c->lastOnCaller && p + 1 == passes;
        const hipStream_t hs = multi ? (defer ? (lastOnCaller ? s : hufS[p % hufStreams]) : c->side) : sideS;
        if (multi && hs != s) {
            HIPCHK(hipEventRecord(c->evDStage[b], s));
            HIPCHK(hipStreamWaitEvent(hs, c->evDStage[b], 0));
        }
        // the deferred sections (kHufFrames frames of one stream type per wave), ahead of the pass's
        // merge: they overlap the next pass's frame decode
        // the last hufWideLast deferred passes: the latency-first decoder (dec_huf_wide_kernel)
        const bool wide = deferP && p + c->hufWideLast >= nDefPasses;
        if (deferP && wide)
            hipLaunchKernelGGL(dec_huf_wide_kernel, dim3((unsigned)(nu * a.G)), dim3(64 * kCoopWaves), 0, hs, a);
        else if (deferP)
            hipLaunchKernelGGL(dec_huf_kernel, dim3((unsigned)(nu * ((a.G + kHufFrames - 1) / kHufFrames))), dim3(64), 0, hs, a);
        // with deferred sections over several passes the merge goes to the third stream behind its
        // pass's sections (so it overlaps the next pass's sections); the buffer is free after it
        hipStream_t ms = hs;
        if (defer && multi && hufStreams < 3 && hs != s) {
            HIPCHK(hipEventRecord(c->evDHuf[b], hs));
            HIPCHK(hipStreamWaitEvent(c->mergeS, c->evDHuf[b], 0));
            ms = c->mergeS;
        }
        if (codec == kCodecVbz) hipLaunchKernelGGL(vbz_merge_kernel, dim3((unsigned)G), dim3(64), 0, ms, a);
        else if (a.lookback)  // few chunks: kMergeRanges single-wave workgroups per chunk
            hipLaunchKernelGGL(dec_merge_lb_kernel, dim3((unsigned)(G * kMergeRanges)), dim3(64), 0, ms, a);
        else hipLaunchKernelGGL(dec_merge_kernel, dim3((unsigned)G), dim3(64), 0, ms, a);
        if (passes > 1) HIPCHK(hipEventRecord(c->evDFree[b], ms));
    }
    HIPCHK(hipGetLastError());
    if (multi && defer && hufStreams == 3) {  // every buffer's last merge (each follows its pass's sections)
        for (size_t b = 0; b < nbuf; b++) HIPCHK(hipStreamWaitEvent(s, c->evDFree[b], 0));
    } else if (multi) {  // the last merge follows every other launch of the call on the side streams
        HIPCHK(hipEventRecord(c->evJoin, defer ? c->mergeS : c->side));
        HIPCHK(hipStreamWaitEvent(s, c->evJoin, 0));
    }
    return PGN_OK;
}

// ---- the large-chunk pass --------------------------------------------------------------------
// A call whose chunks may exceed kPassSamples (maxHint = the caller's bound on the sample counts,
// 0 = unknown) lists them on the scan stream, after the work queued before the call, while the
// batched pass runs (which leaves them UNSUPPORTED); the host reads the list's header and, when it
// is not empty, runs the fused kernel over the listed chunks with slot buffers spaced for the
// largest of them.  Chunks above PGN_MAX_CHUNK_SAMPLES stay UNSUPPORTED.
static bool need_scan(uint32_t maxHint) { return maxHint == 0 || maxHint > kPassSamples; }

// decode calls also list the chunks of the claims pass (claim_scan_kernel), given their blobs
struct ScanBlobs {
    const uint8_t* in;
    const uint64_t* offsets;
    const uint64_t* sizes;
    int nf;
};
static int start_scan(pgn_ctx* c, size_t nchunks, const uint32_t* d_counts, hipStream_t s,
                      const ScanBlobs* blobs = nullptr)
{
    if (nchunks > c->largeListCap) {
        wait_last_host(c);
        (void)hipStreamSynchronize(c->scanStream);
        (void)hipFree(c->largeList);
        (void)hipFree(c->claimList);
        c->largeList = c->claimList = nullptr;
        const size_t m = nchunks < 4096 ? 4096 : nchunks;
        HIPCHK(hipMalloc(&c->largeList, 4 * m));
        HIPCHK(hipMalloc(&c->claimList, 4 * m));
        c->largeListCap = m;
    }
    HIPCHK(hipEventRecord(c->evScanFork, s));
    HIPCHK(hipStreamWaitEvent(c->scanStream, c->evScanFork, 0));
    HIPCHK(hipMemsetAsync(c->largeHdr, 0, 8 * sizeof(uint32_t), c->scanStream));
    unsigned grid = (unsigned)((nchunks + 255) / 256);
    grid = grid > 1024 ? 1024 : grid;
    hipLaunchKernelGGL(large_scan_kernel, dim3(grid), dim3(256), 0, c->scanStream, d_counts, nchunks, c->largeList,
                       c->largeHdr);
    if (blobs)
        hipLaunchKernelGGL(claim_scan_kernel, dim3(grid), dim3(256), 0, c->scanStream, blobs->in, blobs->offsets,
                           blobs->sizes, d_counts, nchunks, blobs->nf, c->claimList, c->largeHdr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->largeHdrHost, c->largeHdr, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->scanStream));
    HIPCHK(hipEventRecord(c->evScan, c->scanStream));
    return PGN_OK;
}

// slot buffers of the large pass: spaced for the largest listed chunk (64 Ki-sample steps, so that
// similar calls reuse them), as many slots as fit kLargeScratchBudget (at least one)
constexpr size_t kLargeScratchBudget = (size_t)8 << 30;
static uint32_t large_cap(uint32_t maxN)
{
    const uint64_t r = ((uint64_t)maxN + 65535u) & ~(uint64_t)65535u;
    return r > PGN_MAX_CHUNK_SAMPLES ? PGN_MAX_CHUNK_SAMPLES : (uint32_t)r;
}
static int ensure_large_enc(pgn_ctx* c, size_t bytes, size_t epochSlots)
{
    if (bytes > c->largeScratchBytes || epochSlots > c->largeEpochSlots) {
        wait_last_host(c);
        (void)hipFree(c->largeScratch);
        (void)hipFree(c->largeEpochs);
        c->largeScratch = nullptr;
        c->largeEpochs = nullptr;
        c->largeScratchBytes = c->largeEpochSlots = 0;
        HIPCHK(hipMalloc(&c->largeScratch, bytes));
        HIPCHK(hipMalloc(&c->largeEpochs, 4 * epochSlots));
        // fresh tables: tag 0 never matches (as in ensure_enc)
        HIPCHK(hipMemsetAsync(c->largeEpochs, 0, 4 * epochSlots, c->stream));
        HIPCHK(hipMemsetAsync(c->largeScratch, 0, bytes, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->largeScratchBytes = bytes;
        c->largeEpochSlots = epochSlots;
    }
    return PGN_OK;
}
static int ensure_large_dec(pgn_ctx* c, size_t bytes)
{
    if (bytes > c->largeDecScratchBytes) {
        wait_last_host(c);
        (void)hipFree(c->largeDecScratch);
        c->largeDecScratch = nullptr;
        c->largeDecScratchBytes = 0;
        HIPCHK(hipMalloc(&c->largeDecScratch, bytes));
        c->largeDecScratchBytes = bytes;
    }
    return PGN_OK;
}
static size_t large_slots(pgn_ctx* c, uint32_t count, size_t slotBytes, size_t fusedMax)
{
    size_t slots = count < fusedMax ? count : fusedMax;
    if (slots * slotBytes > kLargeScratchBudget) slots = kLargeScratchBudget / slotBytes;
    return slots ? slots : 1;
}

static int finish_scan(pgn_ctx* c, uint32_t& count, uint32_t& maxN, uint32_t* maxAll = nullptr)
{
    HIPCHK(hipEventSynchronize(c->evScan));
    count = c->largeHdrHost[0];
    maxN = c->largeHdrHost[1];
    if (maxAll) *maxAll = c->largeHdrHost[3];
    return PGN_OK;
}
// the batched decode's per-chunk sample bound: a multiple of 4096 covering every chunk of the call
static uint32_t call_cap(uint32_t maxN)
{
    const uint32_t r = (maxN + 4095u) & ~4095u;
    return r < 4096u ? 4096u : (r > kPassSamples ? kPassSamples : r);
}

static int launch_large_encode(pgn_ctx* c, int codec, uint32_t count, uint32_t maxN, size_t nchunks,
                               const int16_t* d_samples, const uint64_t* d_sample_offsets,
                               const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                               const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                               hipStream_t s)
{
    const uint32_t capN = large_cap(maxN);
    const size_t sb = enc_slot_bytes(capN);
    const size_t slots = large_slots(c, count, sb, c->encFusedSlotsMax);
    int rc = ensure_large_enc(c, sb * slots, slots);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(c->largeHdr + 2, 0, sizeof(uint32_t), s));
    EncArgs a{};
    a.nchunks = count;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.out = d_out;
    a.outOffsets = d_out_offsets;
    a.outCaps = d_out_caps;
    a.outSizes = d_out_sizes;
    a.status = d_status;
    a.stats = d_stats;
    a.slotScratch = c->largeScratch;
    a.slotBytes = sb;
    a.epochs = c->largeEpochs;
    a.prof = c->prof;
    a.queue = c->largeHdr + 2;
    a.capN = capN;
    a.list = c->largeList;
    (void)nchunks;
    return launch_enc_chunks(codec, a, slots, s);
}

static int launch_large_decode(pgn_ctx* c, int codec, uint32_t count, uint32_t maxN, const uint8_t* d_in,
                               const uint64_t* d_in_offsets, const uint64_t* d_in_sizes, int16_t* d_samples,
                               const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, int32_t* d_status,
                               hipStream_t s)
{
    const uint32_t capN = large_cap(maxN);
    const size_t sb = dec_slot_bytes(capN);
    const size_t slots = large_slots(c, count, sb, c->decFusedSlotsMax);
    int rc = ensure_large_dec(c, sb * slots);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(c->largeHdr + 2, 0, sizeof(uint32_t), s));
    DecArgs a{};
    a.nchunks = count;
    a.in = d_in;
    a.inOffsets = d_in_offsets;
    a.inSizes = d_in_sizes;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.status = d_status;
    a.slotScratch = c->largeDecScratch;
    a.slotBytes = sb;
    a.prof = c->prof ? c->prof + kPhases : nullptr;
    a.queue = c->largeHdr + 2;
    a.capN = capN;
    a.list = c->largeList;
    return launch_dec_chunks(codec, a, slots, s);
}

// The claims pass: the listed chunks (list: device, count entries) decoded as the reference decodes
// them -- every frame into exactly its content-size claim, in an intermediate of the claims' sum
// (maxSum: the largest listed sum; above kClaimPassMax the chunk is PGN_ERR_ALLOC) -- then merged;
// their statuses and samples replace the batched pass's.  The fused kernel, slot scratch of the
// large pass (ordered after it on the stream).
static int launch_claims_decode(pgn_ctx* c, int codec, uint32_t count, uint64_t maxSum, const uint32_t* list,
                                const uint8_t* d_in, const uint64_t* d_in_offsets, const uint64_t* d_in_sizes,
                                int16_t* d_samples, const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts,
                                int32_t* d_status, hipStream_t s)
{
    const uint64_t cap = (maxSum < kClaimPassMax ? maxSum : kClaimPassMax) + kVbzPadding;
    const size_t sb = dec_layout().bytes + align_up(cap + 64, 256);
    const size_t slots = large_slots(c, count, sb, c->decFusedSlotsMax);
    int rc = ensure_large_dec(c, sb * slots);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(c->largeHdr + 2, 0, sizeof(uint32_t), s));
    DecArgs a{};
    a.nchunks = count;
    a.in = d_in;
    a.inOffsets = d_in_offsets;
    a.inSizes = d_in_sizes;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.status = d_status;
    a.slotScratch = c->largeDecScratch;
    a.slotBytes = sb;
    a.prof = c->prof ? c->prof + kPhases : nullptr;
    a.queue = c->largeHdr + 2;
    a.capN = PGN_MAX_CHUNK_SAMPLES;
    a.list = list;
    a.interBytes = cap;
    return launch_dec_chunks(codec, a, slots, s);
}

// The claims pass for chunks of a host-memory call (the blobs are in host memory too): the chunks
// among [0, n) whose status came back PGN_ERR_UNSUPPORTED are listed on the host from their own bytes
// (the device arrays describe the same chunks); then the pass runs and the call waits for it.
static int claims_from_host(pgn_ctx* c, int codec, size_t n, const int32_t* status, const uint32_t* counts,
                            const uint8_t* const* blobs, const uint64_t* blobLens, const uint8_t* d_in,
                            const uint64_t* d_in_offsets, const uint64_t* d_in_sizes, int16_t* d_samples,
                            const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, int32_t* d_status,
                            hipStream_t s)
{
    uint32_t idx[kPcMaxReqs];
    uint32_t k = 0;
    uint64_t maxSum = 0;
    const int nf = codec_frames(codec);
    for (size_t i = 0; i < n && k < (uint32_t)kPcMaxReqs; i++) {
        uint64_t sum = 0;
        if (status[i] != PGN_ERR_UNSUPPORTED || counts[i] > PGN_MAX_CHUNK_SAMPLES) continue;
        if (!claims_pass_chunk(blobs[i], blobLens[i], nf, counts[i], &sum)) continue;
        idx[k++] = (uint32_t)i;
        maxSum = sum > maxSum ? sum : maxSum;
    }
    if (k == 0) return PGN_OK;
    if (!c->claimList || c->largeListCap < kPcMaxReqs) {
        const size_t m = c->largeListCap > 4096 ? c->largeListCap : 4096;
        (void)hipFree(c->claimList);
        (void)hipFree(c->largeList);
        c->claimList = c->largeList = nullptr;
        HIPCHK(hipMalloc(&c->largeList, 4 * m));
        HIPCHK(hipMalloc(&c->claimList, 4 * m));
        c->largeListCap = m;
    }
    HIPCHK(hipMemcpyAsync(c->claimList, idx, 4 * k, hipMemcpyHostToDevice, s));
    const int rc = launch_claims_decode(c, codec, k, maxSum, c->claimList, d_in, d_in_offsets, d_in_sizes, d_samples,
                                        d_sample_offsets, d_sample_counts, d_status, s);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s));
    return PGN_OK;
}

// Every launch sequence on a context: ordered after the previous one (evLast, whatever its stream),
// and recorded as the new last one.  ev[0..1] / ev[2..3] bracket the call's kernels.
static int launch_encode(pgn_ctx* c, int codec, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                         const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                         void* stream, uint32_t maxHint)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (c->haveLast) HIPCHK(hipStreamWaitEvent(s, c->evLast, 0));
    const bool scan = need_scan(maxHint);
    int rc = scan ? start_scan(c, nchunks, d_sample_counts, s) : PGN_OK;
    if (rc == PGN_OK)
        rc = launch_encode_impl(c, codec, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                                d_out_caps, d_out_sizes, d_status, d_stats, s);
    uint32_t count = 0, maxN = 0;
    if (rc == PGN_OK && scan) rc = finish_scan(c, count, maxN);
    if (rc == PGN_OK && count)
        rc = launch_large_encode(c, codec, count, maxN, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out,
                                 d_out_offsets, d_out_caps, d_out_sizes, d_status, d_stats, s);
    if (rc == PGN_OK) {
        HIPCHK(hipEventRecord(c->ev[1], s));
        c->encTimed = true;
    }
    HIPCHK(hipEventRecord(c->evLast, s));
    c->haveLast = true;
    return rc;
}

static int launch_decode(pgn_ctx* c, int codec, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                         const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, int32_t* d_status, void* stream, uint32_t maxHint)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (c->haveLast) HIPCHK(hipStreamWaitEvent(s, c->evLast, 0));
    const bool scan = need_scan(maxHint);
    // The intermediates are spaced for the call's largest chunk when the caller bounds it, else for
    // kPassSamples (the scan then runs beside the batched pass, and the launch stays asynchronous).
    uint32_t capCall = (!scan && maxHint) ? call_cap(maxHint) : kPassSamples;
    uint32_t count = 0, maxN = 0;
    const ScanBlobs blobs{d_in, d_in_offsets, d_in_sizes, codec_frames(codec)};
    int rc = scan ? start_scan(c, nchunks, d_sample_counts, s, &blobs) : PGN_OK;
    // small calls (the per-chunk ones) keep the full capacity: a frame is then decoded up to its own
    // content size, as the reference does, and the chunk ends with its statuses (e.g. "Remaining
    // data" for samples fewer than the frames hold) rather than PGN_ERR_UNSUPPORTED
    if (nchunks <= kCoopMaxChunks) capCall = kPassSamples;
    if (rc == PGN_OK)
        rc = launch_decode_impl(c, codec, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                                d_sample_counts, d_status, s, capCall);
    if (rc == PGN_OK && scan) rc = finish_scan(c, count, maxN);
    if (rc == PGN_OK && count)
        rc = launch_large_decode(c, codec, count, maxN, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                                 d_sample_counts, d_status, s);
    // the chunks whose frames claim more than the passes' intermediates hold (listed by the scan)
    if (rc == PGN_OK && scan && c->largeHdrHost[4])
        rc = launch_claims_decode(c, codec, c->largeHdrHost[4], (uint64_t)c->largeHdrHost[5] << 10, c->claimList, d_in,
                                  d_in_offsets, d_in_sizes, d_samples, d_sample_offsets, d_sample_counts, d_status, s);
    if (rc == PGN_OK) {
        HIPCHK(hipEventRecord(c->ev[3], s));
        c->decTimed = true;
    }
    HIPCHK(hipEventRecord(c->evLast, s));
    c->haveLast = true;
    return rc;
}

static int compress_batch(int codec, pgn_ctx* c, size_t nchunks, const int16_t* d_samples,
                          const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out,
                          const uint64_t* d_out_offsets, const uint64_t* d_out_caps, uint64_t* d_out_sizes,
                          int32_t* d_status, uint64_t* d_stats, void* stream, uint32_t maxHint = 0)
{
    if (!c || !d_samples || !d_sample_offsets || !d_sample_counts || !d_out || !d_out_offsets || !d_out_caps ||
        !d_out_sizes || !d_status)
        return PGN_ERR_INVALID_ARG;
    if (nchunks == 0) return PGN_OK;
    std::lock_guard<std::mutex> g(c->mu);
    return launch_encode(c, codec, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets, d_out_caps,
                         d_out_sizes, d_status, d_stats, stream, maxHint);
}

static int decompress_batch(int codec, pgn_ctx* c, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                            const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                            const uint32_t* d_sample_counts, int32_t* d_status, void* stream, uint32_t maxHint = 0)
{
    if (!c || !d_in || !d_in_offsets || !d_in_sizes || !d_samples || !d_sample_offsets || !d_sample_counts || !d_status)
        return PGN_ERR_INVALID_ARG;
    if (nchunks == 0) return PGN_OK;
    std::lock_guard<std::mutex> g(c->mu);
    return launch_decode(c, codec, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets, d_sample_counts,
                         d_status, stream, maxHint);
}

int pgn_compress_batch_device(pgn_ctx* c, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                              const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                              const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                              void* stream)
{
    return compress_batch(kCodecC5, c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                          d_out_caps, d_out_sizes, d_status, d_stats, stream);
}

int pgn_compress_batch_device_bounded(pgn_ctx* c, uint32_t max_chunk_samples, size_t nchunks, const int16_t* d_samples,
                                      const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out,
                                      const uint64_t* d_out_offsets, const uint64_t* d_out_caps, uint64_t* d_out_sizes,
                                      int32_t* d_status, uint64_t* d_stats, void* stream)
{
    return compress_batch(kCodecC5, c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                          d_out_caps, d_out_sizes, d_status, d_stats, stream, max_chunk_samples ? max_chunk_samples : 1u);
}

int pgn_decompress_batch_device_bounded(pgn_ctx* c, uint32_t max_chunk_samples, size_t nchunks, const uint8_t* d_in,
                                        const uint64_t* d_in_offsets, const uint64_t* d_in_sizes, int16_t* d_samples,
                                        const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts,
                                        int32_t* d_status, void* stream)
{
    return decompress_batch(kCodecC5, c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                            d_sample_counts, d_status, stream, max_chunk_samples ? max_chunk_samples : 1u);
}

int pgn_decompress_batch_device(pgn_ctx* c, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                                const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                                const uint32_t* d_sample_counts, int32_t* d_status, void* stream)
{
    return decompress_batch(kCodecC5, c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                            d_sample_counts, d_status, stream);
}

int pgn_vbz_compress_batch_device(pgn_ctx* c, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                                  const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                                  const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status,
                                  uint64_t* d_stats, void* stream)
{
    return compress_batch(kCodecVbz, c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                          d_out_caps, d_out_sizes, d_status, d_stats, stream);
}

int pgn_vbz_decompress_batch_device(pgn_ctx* c, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                                    const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                                    const uint32_t* d_sample_counts, int32_t* d_status, void* stream)
{
    return decompress_batch(kCodecVbz, c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                            d_sample_counts, d_status, stream);
}

// the pgnano variants by pgn_variant id -> internal codec
static int variant_codec(int variant)
{
    switch (variant) {
    case PGN_VARIANT_C5: return kCodecC5;
    case PGN_VARIANT_C4: return kCodecC4;
    case PGN_VARIANT_C1: return kCodecC1;
    case PGN_VARIANT_C2: return kCodecC2;
    case PGN_VARIANT_C3: return kCodecC3;
    case PGN_VARIANT_VBZ0: return kCodecVbz0;
    default: return -1;
    }
}

int pgn_variant_compress_batch_device(pgn_ctx* c, int variant, size_t nchunks, const int16_t* d_samples,
                                      const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out,
                                      const uint64_t* d_out_offsets, const uint64_t* d_out_caps, uint64_t* d_out_sizes,
                                      int32_t* d_status, uint64_t* d_stats, void* stream)
{
    const int codec = variant_codec(variant);
    if (codec < 0) return PGN_ERR_INVALID_ARG;
    return compress_batch(codec, c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets,
                          d_out_caps, d_out_sizes, d_status, d_stats, stream);
}

int pgn_variant_decompress_batch_device(pgn_ctx* c, int variant, size_t nchunks, const uint8_t* d_in,
                                        const uint64_t* d_in_offsets, const uint64_t* d_in_sizes, int16_t* d_samples,
                                        const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts,
                                        int32_t* d_status, void* stream)
{
    const int codec = variant_codec(variant);
    if (codec < 0) return PGN_ERR_INVALID_ARG;
    return decompress_batch(codec, c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets,
                            d_sample_counts, d_status, stream);
}

}  // extern "C"

static int bounded_codec(int codec)
{
    return codec == PGN_POD5_CODEC_VBZ ? (int)kCodecVbz : variant_codec(codec);
}

int pgn_compress_batch_bounded(pgn_ctx* c, int codec, uint32_t max_samples, size_t nchunks, const int16_t* d_samples,
                               const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out,
                               const uint64_t* d_out_offsets, const uint64_t* d_out_caps, uint64_t* d_out_sizes,
                               int32_t* d_status, uint64_t* d_stats, void* stream)
{
    const int k = bounded_codec(codec);
    if (k < 0) return PGN_ERR_INVALID_ARG;
    return compress_batch(k, c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets, d_out_caps,
                          d_out_sizes, d_status, d_stats, stream, max_samples);
}

int pgn_decompress_batch_bounded(pgn_ctx* c, int codec, uint32_t max_samples, size_t nchunks, const uint8_t* d_in,
                                 const uint64_t* d_in_offsets, const uint64_t* d_in_sizes, int16_t* d_samples,
                                 const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, int32_t* d_status,
                                 void* stream)
{
    const int k = bounded_codec(codec);
    if (k < 0) return PGN_ERR_INVALID_ARG;
    return decompress_batch(k, c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets, d_sample_counts,
                            d_status, stream, max_samples);
}

extern "C" {

#ifdef PGN_DEBUG_HUF
// diagnostic build only: the Huffman decoder's record buffer (count, then records of 8 words)
int pgn_debug_huf_dump(uint32_t* out, size_t nwords)
{
    uint32_t cnt = 0;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(gHufDbgN), 4));
    out[0] = cnt;
    size_t m = cnt < (1u << 18) ? cnt : (1u << 18);
    if (m > nwords - 1) m = nwords - 1;
    HIPCHK(hipMemcpyFromSymbol(out + 1, HIP_SYMBOL(gHufDbg), 4 * m));
    return PGN_OK;
}
#endif

int pgn_debug_phase_cycles(pgn_ctx* c, uint64_t* out, int n)
{
    if (!c || !out || n < 2 * kPhases) return PGN_ERR_INVALID_ARG;
    const int m = n < kProfWords ? n : kProfWords;
    if (!c->prof) {
        memset(out, 0, sizeof(uint64_t) * m);
        return PGN_OK;
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->prof, sizeof(uint64_t) * m, hipMemcpyDeviceToHost));
    return PGN_OK;
}

// Diagnostics: the per-stream decode records {frame offset, length, content size, offset, result}
// of the first n chunks of the last decode pass (24 bytes each, 5 per chunk).
int pgn_debug_decode_units(pgn_ctx* c, void* out, size_t nchunks)
{
    if (!c || !out) return PGN_ERR_INVALID_ARG;
    if (!c->lastUnits || nchunks > c->lastG) return PGN_ERR_INVALID_ARG;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->lastUnits, nchunks * kStreams * sizeof(DecUnit), hipMemcpyDeviceToHost));
    return PGN_OK;
}

const char* pgn_ctx_kernels(pgn_ctx* c, int direction)
{
    if (!c) return "";
    if (direction == 0)
        return c->encStaged ? "enc_split_kernel + enc_zstd_kernel + enc_assemble_kernel" : "enc_chunk_kernel<C5>";
    if (!c->decStaged) return "dec_chunk_kernel<C5>";
    return c->lastDeferred ? "dec_parse_kernel + dec_zstd_kernel + dec_huf_kernel + dec_merge_kernel"
                           : "dec_parse_kernel + dec_zstd_kernel + dec_merge_kernel";
}

float pgn_ctx_last_encode_ms(pgn_ctx* c)
{
    if (!c || !c->encTimed) return -1.f;
    float ms = -1.f;
    if (hipEventSynchronize(c->ev[1]) != hipSuccess) return -1.f;
    if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) != hipSuccess) return -1.f;
    return ms;
}
float pgn_ctx_last_decode_ms(pgn_ctx* c)
{
    if (!c || !c->decTimed) return -1.f;
    float ms = -1.f;
    if (hipEventSynchronize(c->ev[3]) != hipSuccess) return -1.f;
    if (hipEventElapsedTime(&ms, c->ev[2], c->ev[3]) != hipSuccess) return -1.f;
    return ms;
}

int pgn_synth_reads_device(pgn_ctx* c, size_t nreads, uint64_t seed, uint64_t first_read, uint64_t read_stride,
                           int16_t* d_samples,
                           const uint64_t* d_offsets, const uint32_t* d_counts, uint32_t pq, int32_t mean, int32_t lsd,
                           int32_t nsd, void* stream)
{
    if (!c || !d_samples || !d_offsets || !d_counts) return PGN_ERR_INVALID_ARG;
    if (nreads == 0) return PGN_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // task prefix sums (host-side scan over a device copy of the counts: simple and off the timed path)
    uint32_t* hc = (uint32_t*)malloc(4 * nreads);
    uint64_t* hs = (uint64_t*)malloc(8 * (nreads + 1));
    if (!hc || !hs) { free(hc); free(hs); return PGN_ERR_INVALID_ARG; }
    HIPCHK(hipMemcpyAsync(hc, d_counts, 4 * nreads, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    hs[0] = 0;
    for (size_t r = 0; r < nreads; r++) hs[r + 1] = hs[r] + (hc[r] + 63u) / 64u;
    uint64_t* dts = nullptr;
    HIPCHK(hipMallocAsync((void**)&dts, 8 * (nreads + 1), s));
    HIPCHK(hipMemcpyAsync(dts, hs, 8 * (nreads + 1), hipMemcpyHostToDevice, s));
    SynthArgs a{nreads, seed, first_read, read_stride ? read_stride : 1, d_samples, d_offsets, d_counts, pq, mean, lsd, nsd};
    uint64_t tasks = hs[nreads];
    unsigned grid = (unsigned)((tasks + 255) / 256);
    if (grid > 65536) grid = 65536;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(256), 0, s, a, tasks, (const uint64_t*)dts);
    HIPCHK(hipGetLastError());
    HIPCHK(hipFreeAsync(dts, s));
    HIPCHK(hipStreamSynchronize(s));
    free(hc);
    free(hs);
    return PGN_OK;
}

// ---- host-memory per-chunk entry points (the plugin surface) --------------------------------
static int ensure_stage(pgn_ctx* c, size_t bytes)
{
    if (bytes <= c->stageBytes) return PGN_OK;
    wait_last_host(c);
    (void)hipFree(c->stage);
    if (c->hstage) (void)hipHostFree(c->hstage);
    c->stage = nullptr;
    c->hstage = nullptr;
    c->stageBytes = 0;
    size_t b = align_up(bytes, 1 << 20);
    HIPCHK(hipMalloc(&c->stage, b));
    HIPCHK(hipHostMalloc((void**)&c->hstage, b, hipHostMallocDefault));
    HIPCHK(hipHostGetDevicePointer((void**)&c->hstageDev, c->hstage, 0));
    c->stageBytes = b;
    return PGN_OK;
}

struct StageHdr {
    uint64_t off0, cnt0pad, outOff, outCap, outSize, inOff, inSize;
    uint32_t count;
    int32_t status;
    uint64_t stats[PGN_STATS_PER_CHUNK];
};

// One chunk from host memory: header and samples staged in the pinned mirror and uploaded in one
// copy; the kernels write the blob, its size, status and stats straight into the pinned mirror
// (no copies back: the call's tail is the kernels and one wait); the blob leaves it by memcpy.
static int compress_signal_one(int codec, pgn_ctx* c, const int16_t* samples, size_t n, uint8_t* dst, size_t cap,
                               size_t* out_size)
{
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    const size_t hdrB = 256, inB = align_up(2 * n + 16, 256);
    int rc = ensure_stage(c, hdrB + inB + cap + 64);
    if (rc) return rc;
    uint8_t* dh = c->stage;
    uint8_t* din = c->stage + hdrB;
    uint8_t* hout = c->hstageDev + hdrB + inB;  // the blob, written by the kernels into host memory
    StageHdr* hh = (StageHdr*)c->hstage;
    StageHdr* hd = (StageHdr*)c->hstageDev;     // the same header, the outputs written by the kernels
    *hh = StageHdr{};
    hh->outCap = cap;
    hh->count = (uint32_t)n;
    if (n) memcpy(c->hstage + hdrB, samples, 2 * n);
    HIPCHK(hipMemcpyAsync(dh, c->hstage, hdrB + 2 * n, hipMemcpyHostToDevice, c->stream));
    StageHdr* d = (StageHdr*)dh;
    rc = launch_encode(c, codec, 1, (const int16_t*)din, &d->off0, &d->count, hout, &d->outOff, &d->outCap,
                       &hd->outSize, &hd->status, hd->stats, c->stream, n ? (uint32_t)n : 1u);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    *out_size = (size_t)hh->outSize;
    if (hh->status != PGN_OK) return hh->status;
    memcpy(dst, c->hstage + hdrB + inB, (size_t)hh->outSize);
    return PGN_OK;
}

static int decompress_signal_one(int codec, pgn_ctx* c, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    const size_t hdrB = 256, inB = align_up(len + 16, 256);
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = ensure_stage(c, hdrB + inB + 2 * n + 64);
    if (rc) return rc;
    uint8_t* dh = c->stage;
    uint8_t* din = c->stage + hdrB;
    int16_t* hout = (int16_t*)(c->hstageDev + hdrB + inB);  // the samples, written by the kernels into host memory
    StageHdr* hh = (StageHdr*)c->hstage;
    StageHdr* hd = (StageHdr*)c->hstageDev;
    *hh = StageHdr{};
    hh->inSize = len;
    hh->count = (uint32_t)n;
    if (len) memcpy(c->hstage + hdrB, src, len);
    HIPCHK(hipMemcpyAsync(dh, c->hstage, hdrB + len, hipMemcpyHostToDevice, c->stream));
    StageHdr* d = (StageHdr*)dh;
    rc = launch_decode(c, codec, 1, din, &d->inOff, &d->inSize, hout, &d->off0, &d->count, &hd->status, c->stream,
                       n ? (uint32_t)n : 1u);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (hh->status == PGN_ERR_UNSUPPORTED) {  // frames claiming more than the intermediate: the claims pass
        const uint8_t* bl = c->hstage + hdrB;
        const uint64_t ln = len;
        rc = claims_from_host(c, codec, 1, &hh->status, &hh->count, &bl, &ln, din, &d->inOff, &d->inSize, hout, &d->off0,
                              &d->count, &hd->status, c->stream);
        if (rc) return rc;
    }
    if (hh->status != PGN_OK) return hh->status;
    if (n) memcpy(dst, c->hstage + hdrB + inB, 2 * n);
    return PGN_OK;
}

// An arena's per-request arrays (kPcHdr bytes at its start; index = the request's place in the
// batch order): the kernels read the device mirror's copy and write the results into pinned memory.
struct PcHdr {
    uint64_t off0[kPcMaxReqs];     // sample offset (elements): encode from the inputs, decode from the outputs
    uint32_t cnt[kPcMaxReqs];
    uint64_t outOff[kPcMaxReqs];   // encode: blob offset in the outputs
    uint64_t outCap[kPcMaxReqs];
    uint64_t inOff[kPcMaxReqs];    // decode: blob offset in the inputs
    uint64_t inSize[kPcMaxReqs];
    uint64_t outSize[kPcMaxReqs];  // results
    int32_t status[kPcMaxReqs];
    uint64_t stats[kPcMaxReqs * PGN_STATS_PER_CHUNK];
};
static_assert(sizeof(PcHdr) <= kPcHdr, "per-request arrays");

static int pc_init(pgn_ctx* c)
{
    HIPCHK(hipSetDevice(c->device));
    for (PcArena& A : c->pcA) {
        HIPCHK(hipHostMalloc((void**)&A.h, kPcHdr + kPcInCap + kPcOutCap, hipHostMallocDefault));
        HIPCHK(hipHostGetDevicePointer((void**)&A.hDev, A.h, 0));
        HIPCHK(hipMalloc(&A.d, kPcHdr + kPcInCap));
    }
    return PGN_OK;
}

// One arena's requests as one batch per (direction, codec) group, each group a batched launch over
// the arena's arrays; one upload, one wait.  Called by the leader without pcMu.
static void pc_run(pgn_ctx* c, PcArena& A)
{
    const int k = A.nreq;
    PcReq* ord[kPcMaxReqs];
    for (int i = 0; i < k; i++) ord[i] = A.reqs[i];
    std::stable_sort(ord, ord + k, [](const PcReq* x, const PcReq* y) {
        return x->dir * 16 + x->codec < y->dir * 16 + y->codec;
    });
    PcHdr* hh = (PcHdr*)A.h;
    for (int i = 0; i < k; i++) {
        const PcReq& r = *ord[i];
        hh->cnt[i] = r.n;
        hh->status[i] = -1;
        hh->outSize[i] = 0;
        if (r.dir == 0) {
            hh->off0[i] = r.inOff / 2;
            hh->outOff[i] = r.outOff;
            hh->outCap[i] = r.cap;
        } else {
            hh->off0[i] = r.outOff / 2;
            hh->inOff[i] = r.inOff;
            hh->inSize[i] = r.inBytes;
        }
    }
    const PcHdr* dh = (const PcHdr*)A.d;  // the device mirror of the arrays
    PcHdr* ho = (PcHdr*)A.hDev;           // results straight into pinned memory
    uint8_t* const inD = A.d + kPcHdr;
    uint8_t* const outH = A.hDev + kPcHdr + kPcInCap;
    int rc = PGN_OK;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess ||
            hipMemcpyAsync(A.d, A.h, kPcHdr + A.inUsed, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            rc = PGN_ERR_HIP;
        for (int i0 = 0; rc == PGN_OK && i0 < k;) {
            int i1 = i0;
            uint32_t maxN = 1;
            while (i1 < k && ord[i1]->dir == ord[i0]->dir && ord[i1]->codec == ord[i0]->codec) {
                maxN = ord[i1]->n > maxN ? ord[i1]->n : maxN;
                i1++;
            }
            const size_t m = (size_t)(i1 - i0);
            if (ord[i0]->dir == 0)
                rc = launch_encode(c, ord[i0]->codec, m, (const int16_t*)inD, dh->off0 + i0, dh->cnt + i0, outH,
                                   dh->outOff + i0, dh->outCap + i0, ho->outSize + i0, ho->status + i0,
                                   ho->stats + (size_t)i0 * PGN_STATS_PER_CHUNK, c->stream, maxN);
            else
                rc = launch_decode(c, ord[i0]->codec, m, inD, dh->inOff + i0, dh->inSize + i0, (int16_t*)outH,
                                   dh->off0 + i0, dh->cnt + i0, ho->status + i0, c->stream, maxN);
            i0 = i1;
        }
        if (hipStreamSynchronize(c->stream) != hipSuccess && rc == PGN_OK) rc = PGN_ERR_HIP;
        // decode chunks whose frames claim more than the batch's intermediates: the claims pass
        for (int i0 = 0; rc == PGN_OK && i0 < k;) {
            int i1 = i0;
            while (i1 < k && ord[i1]->dir == ord[i0]->dir && ord[i1]->codec == ord[i0]->codec) i1++;
            if (ord[i0]->dir == 1) {
                const uint8_t* bl[kPcMaxReqs];
                uint64_t ln[kPcMaxReqs];
                for (int i = i0; i < i1; i++) {
                    bl[i - i0] = A.h + kPcHdr + ord[i]->inOff;
                    ln[i - i0] = ord[i]->inBytes;
                }
                rc = claims_from_host(c, ord[i0]->codec, (size_t)(i1 - i0), hh->status + i0, hh->cnt + i0, bl, ln, inD,
                                      dh->inOff + i0, dh->inSize + i0, (int16_t*)outH, dh->off0 + i0, dh->cnt + i0,
                                      ho->status + i0, c->stream);
            }
            i0 = i1;
        }
    }
    for (int i = 0; i < k; i++) {
        PcReq& r = *ord[i];
        r.rc = rc != PGN_OK ? rc : hh->status[i];
        r.outSize = hh->outSize[i];
    }
}

enum { kPcExclusive = 1000 };  // the call runs on its own (too large for an arena, or no arenas)

// A per-chunk host call through the arenas (see PcArena).  Returns the call's status, or
// kPcExclusive when it should run by itself.
static int pc_call(pgn_ctx* c, PcReq& r)
{
    const size_t inB = align_up(r.inBytes + 16, 256), outB = align_up(r.outBytes + 64, 256);
    if (inB > kPcInCap || outB > kPcOutCap) return kPcExclusive;
    std::unique_lock<std::mutex> lk(c->pcMu);
    if (c->pcReady == 0) c->pcReady = pc_init(c) == PGN_OK ? 1 : -1;
    if (c->pcReady < 0) return kPcExclusive;
    PcArena* A = nullptr;
    while (true) {  // join the open arena when it has room
        if (c->pcOpen >= 0) {
            PcArena& O = c->pcA[c->pcOpen];
            if (O.nreq < kPcMaxReqs && O.inUsed + inB <= kPcInCap && O.outUsed + outB <= kPcOutCap) {
                A = &O;
                break;
            }
        }
        c->pcCv.wait(lk);
    }
    const int ai = (int)(A - c->pcA);
    r.inOff = A->inUsed;
    r.outOff = A->outUsed;
    A->inUsed += inB;
    A->outUsed += outB;
    A->reqs[A->nreq++] = &r;
    A->unstaged++;
    r.done = false;
    lk.unlock();
    if (r.inBytes) memcpy(A->h + kPcHdr + r.inOff, r.in, r.inBytes);
    lk.lock();
    if (--A->unstaged == 0) c->pcCv.notify_all();
    while (!r.done) {
        if (!c->pcBusy && A->state == 0) {  // lead: run this arena (it holds this call)
            c->pcBusy = true;
            A->state = 1;
            PcArena& B = c->pcA[1 - ai];
            c->pcOpen = (B.state == 0 && B.nreq == 0) ? 1 - ai : -1;  // new calls fill the other arena
            c->pcCv.notify_all();
            while (A->unstaged) c->pcCv.wait(lk);
            lk.unlock();
            pc_run(c, *A);
            lk.lock();
            A->state = 2;
            A->readers = A->nreq;
            for (int i = 0; i < A->nreq; i++) A->reqs[i]->done = true;
            c->pcBusy = false;
            c->pcCv.notify_all();
        } else {
            c->pcCv.wait(lk);
        }
    }
    lk.unlock();
    const uint8_t* res = A->h + kPcHdr + kPcInCap + r.outOff;
    if (r.rc == PGN_OK) {
        if (r.dir == 0) memcpy(r.dst, res, (size_t)r.outSize);
        else if (r.n) memcpy(r.dst, res, 2 * (size_t)r.n);
    }
    lk.lock();
    if (--A->readers == 0) {  // the arena is idle again
        A->state = 0;
        A->nreq = 0;
        A->inUsed = A->outUsed = 0;
        if (c->pcOpen < 0) c->pcOpen = ai;
        c->pcCv.notify_all();
    }
    return r.rc;
}

// The blob bytes an encode call can need: its five frames (each at most ZSTD_COMPRESSBOUND of its
// stream, the streams together at most 3.75 n bytes; VBZ: one frame of ~2.13 n) and their prefixes.
static size_t pc_enc_out_bytes(size_t n, size_t cap)
{
    const size_t b = 4 * n + 4096;
    return cap < b ? cap : b;
}

static int compress_signal(int codec, pgn_ctx* c, const int16_t* samples, size_t n, uint8_t* dst, size_t cap,
                           size_t* out_size)
{
    if (!c || (!samples && n) || !dst || !out_size) return PGN_ERR_INVALID_ARG;
    if (n > PGN_MAX_CHUNK_SAMPLES) return PGN_ERR_UNSUPPORTED;
    PcReq r{};
    r.dir = 0;
    r.codec = codec;
    r.in = samples;
    r.inBytes = 2 * n;
    r.n = (uint32_t)n;
    r.dst = dst;
    r.cap = cap;
    r.outBytes = pc_enc_out_bytes(n, cap);
    const int rc = pc_call(c, r);
    if (rc == kPcExclusive) return compress_signal_one(codec, c, samples, n, dst, cap, out_size);
    *out_size = (size_t)r.outSize;
    return rc;
}

static int decompress_signal(int codec, pgn_ctx* c, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    if (!c || (!src && len) || (!dst && n)) return PGN_ERR_INVALID_ARG;
    if (n > PGN_MAX_CHUNK_SAMPLES) return PGN_ERR_UNSUPPORTED;
    PcReq r{};
    r.dir = 1;
    r.codec = codec;
    r.in = src;
    r.inBytes = len;
    r.n = (uint32_t)n;
    r.dst = dst;
    r.outBytes = 2 * n;
    const int rc = pc_call(c, r);
    if (rc == kPcExclusive) return decompress_signal_one(codec, c, src, len, dst, n);
    return rc;
}

int pgn_compress_signal(pgn_ctx* c, const int16_t* samples, size_t n, uint8_t* dst, size_t cap, size_t* out_size)
{
    return compress_signal(kCodecC5, c, samples, n, dst, cap, out_size);
}

int pgn_decompress_signal(pgn_ctx* c, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    return decompress_signal(kCodecC5, c, src, len, dst, n);
}

size_t pgn_vbz_compressed_signal_max_size(size_t n)
{
    return z1::compress_bound((size_t)svb_key_length((uint32_t)n) + 2 * n);
}

int pgn_vbz_compress_signal(pgn_ctx* c, const int16_t* samples, size_t n, uint8_t* dst, size_t cap, size_t* out_size)
{
    return compress_signal(kCodecVbz, c, samples, n, dst, cap, out_size);
}

int pgn_vbz_decompress_signal(pgn_ctx* c, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    return decompress_signal(kCodecVbz, c, src, len, dst, n);
}

int pgn_variant_compress_signal(pgn_ctx* c, int variant, const int16_t* samples, size_t n, uint8_t* dst, size_t cap,
                                size_t* out_size)
{
    const int codec = variant_codec(variant);
    if (codec < 0) return PGN_ERR_INVALID_ARG;
    return compress_signal(codec, c, samples, n, dst, cap, out_size);
}

int pgn_variant_decompress_signal(pgn_ctx* c, int variant, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    const int codec = variant_codec(variant);
    if (codec < 0) return PGN_ERR_INVALID_ARG;
    return decompress_signal(codec, c, src, len, dst, n);
}

static pgn_ctx* g_default = nullptr;
static std::mutex g_default_mu;

static int default_ctx(pgn_ctx** c)
{
    std::lock_guard<std::mutex> g(g_default_mu);
    if (!g_default) {
        const int rc = pgn_ctx_create(0, &g_default);
        if (rc) return rc;
    }
    *c = g_default;
    return PGN_OK;
}

// The pod5 C-API wrappers (c_api.cpp:1183-1253): compress into a buffer of the codec's maximum size,
// then check the caller's buffer ("Compressed signal size (..) is greater than provided buffer size").
static int capi_compress(int codec, const int16_t* signal, size_t signal_size, char* out, size_t* inout_size)
{
    if (!signal || !out || !inout_size) return PGN_ERR_INVALID_ARG;
    pgn_ctx* c = nullptr;
    int rc = default_ctx(&c);
    if (rc) return rc;
    // pgnano::compress_signal allocates compressed_signal_max_size(n) (pgnano.cpp:66-68), pod5's
    // VBZ compress_signal pod5::compressed_signal_max_size(n) (signal_compression.cpp:21-35) ...
    const size_t cap = codec == kCodecVbz ? pgn_vbz_compressed_signal_max_size(signal_size)
                                          : pgn_compressed_signal_max_size(signal_size);
    uint8_t* tmp = (uint8_t*)malloc(cap);
    if (!tmp) return PGN_ERR_INVALID_ARG;
    size_t sz = 0;
    rc = compress_signal(codec, c, signal, signal_size, tmp, cap, &sz);
    if (rc == PGN_OK) {
        // ... then c_api.cpp:1240-1250 checks the caller's buffer
        if (sz > *inout_size) {
            rc = PGN_ERR_DST_TOO_SMALL;
        } else {
            memcpy(out, tmp, sz);
            *inout_size = sz;
        }
    }
    free(tmp);
    return rc;
}

int pgn_pinanoraw_compress_signal(const int16_t* signal, size_t signal_size, char* out, size_t* inout_size)
{
    return capi_compress(kCodecC5, signal, signal_size, out, inout_size);
}

int pgn_pod5_vbz_compress_signal(const int16_t* signal, size_t signal_size, char* out, size_t* inout_size)
{
    return capi_compress(kCodecVbz, signal, signal_size, out, inout_size);
}

int pgn_pod5_vbz_decompress_signal(const char* compressed, size_t compressed_size, size_t sample_count, short* out)
{
    if (!compressed || !out) return PGN_ERR_INVALID_ARG;  // check_not_null / check_output_pointer_not_null
    pgn_ctx* c = nullptr;
    const int rc = default_ctx(&c);
    if (rc) return rc;
    return decompress_signal(kCodecVbz, c, (const uint8_t*)compressed, compressed_size, (int16_t*)out, sample_count);
}

}  // extern "C"
