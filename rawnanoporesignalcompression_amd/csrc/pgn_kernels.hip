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

#include <mutex>

#include "../../include/pgnano_hip.h"
#include "pgn_c5.h"
#include "pgn_zdec.h"
#include "pgn_zenc.h"

namespace pgn {

constexpr uint32_t kMaxSamples = PGN_MAX_CHUNK_SAMPLES;
constexpr uint32_t kMaxStream = kMaxSamples;            // largest C5 stream (M/Llow/Lhigh <= n)
constexpr uint32_t kMaxEncSeq = kMaxStream / 4 + 2;      // every match covers >= 4 bytes
constexpr uint32_t kMaxDecSeq = kMaxStream / 3 + 2;      // any valid block: matches >= 3 bytes

__host__ __device__ constexpr size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---------------------------------------------------------------------------------------------
// Scratch window of one encode slot
// ---------------------------------------------------------------------------------------------
struct EncLayout {
    size_t K, S, M, Ll, Lh, ht, lit, seqs, codes, seqSection, seqWork, frameTmp, bytes;
};
__host__ __device__ inline EncLayout enc_layout()
{
    EncLayout l{};
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o = align_up(o + n + 64, 256); return r; };
    l.K = take(kMaxSamples / 4 + 1);
    l.S = take(kMaxSamples / 2 + 1);
    l.M = take(kMaxStream);
    l.Ll = take(kMaxStream);
    l.Lh = take(kMaxStream);
    l.ht = take((size_t)4 << 15);
    l.lit = take(kMaxStream);
    l.seqs = take(sizeof(z1::Seq) * kMaxEncSeq);
    l.codes = take(3 * (size_t)kMaxEncSeq);
    l.seqSection = take(16 + 10 * (size_t)kMaxEncSeq + 1024);
    l.seqWork = take(sizeof(z1::SeqWork));
    l.frameTmp = take(z1::compress_bound(kMaxStream) + 64);
    l.bytes = o;
    return l;
}

struct DecLayout {
    size_t inter, lit, seqs, tables, bytes;
};
constexpr size_t kInterCap = (size_t)5 * kMaxStream;
__host__ __device__ inline DecLayout dec_layout()
{
    DecLayout l{};
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o = align_up(o + n + 64, 256); return r; };
    l.inter = take(kInterCap);
    l.lit = take(kMaxStream);
    l.seqs = take(12 * (size_t)kMaxDecSeq);
    l.tables = take(3 * sizeof(z1::FseDTable));
    l.bytes = o;
    return l;
}

// ---------------------------------------------------------------------------------------------
// Encode
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
    uint8_t* scratch;
    size_t slotBytes;
    uint32_t* epochs;
    uint64_t* prof;
};

__global__ __launch_bounds__(64) void c5_encode_kernel(EncArgs a)
{
    __shared__ EncLds L;
    const int lane = lane_id();
    const EncLayout lay = enc_layout();
    uint8_t* base = a.scratch + (size_t)blockIdx.x * a.slotBytes;
    C5Streams st;
    st.K = base + lay.K;
    st.S = base + lay.S;
    st.M = base + lay.M;
    st.Ll = base + lay.Ll;
    st.Lh = base + lay.Lh;
    uint8_t* streams[5] = {st.K, st.S, st.M, st.Ll, st.Lh};
    EncScratch S;
    S.ht = (uint32_t*)(base + lay.ht);
    S.seqs = (z1::Seq*)(base + lay.seqs);
    S.codes = base + lay.codes;
    S.lit = base + lay.lit;
    S.seqSection = base + lay.seqSection;
    S.seqWork = (z1::SeqWork*)(base + lay.seqWork);
    S.maxSeq = kMaxEncSeq;
    uint8_t* frameTmp = base + lay.frameTmp;
    uint32_t epoch = a.epochs[blockIdx.x];
    PhaseProf P;
    P.init(a.prof);

    for (size_t c = blockIdx.x; c < a.nchunks; c += gridDim.x) {
        const uint32_t n = a.sampleCounts[c];
        const uint64_t cap = a.outCaps[c];
        uint8_t* dst = a.out + a.outOffsets[c];
        if (n > kMaxSamples) {
            if (lane == 0) { a.status[c] = PGN_ERR_UNSUPPORTED; a.outSizes[c] = 0; }
            continue;
        }
        uint32_t sizes[5];
        c5_split_wave(a.samples + a.sampleOffsets[c], n, st, sizes, L.split);
        wave_sync();
        P.mark(0);
        uint64_t off = 0, fsz[5];
        bool overflow = false;
        for (int s = 0; s < 5; s++) {
            if (++epoch >= 32768u) {  // tag space exhausted: clear the table once
                for (uint32_t i = (uint32_t)lane; i < (1u << 15); i += 64) S.ht[i] = 0;
                epoch = 1;
                wave_sync();
            }
            const uint64_t hdr = (s < 4) ? 8 : 0;
            const bool direct = !overflow && (off + hdr + z1::compress_bound(sizes[s]) <= cap);
            uint8_t* fdst = direct ? dst + off + hdr : frameTmp;
            fsz[s] = zstd1_compress_wave(fdst, streams[s], sizes[s], L, S, epoch, P);
            if (!direct) {
                if (!overflow && off + hdr + fsz[s] <= cap) wave_copy(dst + off + hdr, frameTmp, fsz[s]);
                else overflow = true;
            }
            if (!overflow && hdr && lane == 0) __builtin_memcpy(dst + off, &fsz[s], 8);
            off += hdr + fsz[s];
            wave_sync();
        }
        if (lane == 0) {
            a.status[c] = overflow ? PGN_ERR_DST_TOO_SMALL : PGN_OK;
            a.outSizes[c] = off;
            if (a.stats) {
                for (int s = 0; s < 5; s++) {
                    a.stats[c * PGN_STATS_PER_CHUNK + s] = sizes[s];
                    a.stats[c * PGN_STATS_PER_CHUNK + 5 + s] = fsz[s];
                }
            }
        }
    }
    if (lane == 0) a.epochs[blockIdx.x] = epoch;
    P.flush();
}

// ---------------------------------------------------------------------------------------------
// Decode
// ---------------------------------------------------------------------------------------------
struct DecArgs {
    size_t nchunks;
    const uint8_t* in;
    const uint64_t* inOffsets;
    const uint64_t* inSizes;
    int16_t* samples;
    const uint64_t* sampleOffsets;
    const uint32_t* sampleCounts;
    int32_t* status;
    uint8_t* scratch;
    size_t slotBytes;
    uint64_t* prof;
};

__device__ inline int c5_decode_chunk(const uint8_t* src, uint64_t len, int16_t* out, uint32_t n,
                                      const DecScratch& S, uint8_t* inter, PhaseProf& P)
{
    const uint8_t* fp[5];
    uint64_t fl[5], cs[5];
    uint64_t pos = 0;
    for (int s = 0; s < 5; s++) {
        if (s < 4) {
            if (pos > len || len - pos < 8) return PGN_ERR_CORRUPT;
            fl[s] = ld64u(src + pos);
            pos += 8;
            if (fl[s] > len - pos) return PGN_ERR_CORRUPT;
        } else {
            fl[s] = len - pos;  // last frame length is implicit (C5.hpp:560)
        }
        fp[s] = src + pos;
        bool ok = false;
        cs[s] = z1::frame_content_size(fp[s], (size_t)fl[s], &ok);
        if (!ok) return PGN_ERR_NOT_ZSTD;
        pos += fl[s];
    }
    uint64_t total = 0;
    for (int s = 0; s < 5; s++) {
        if (cs[s] > kMaxStream) return PGN_ERR_UNSUPPORTED;
        total += cs[s];
    }
    uint64_t off = 0, dres[5];
    for (int s = 0; s < 5; s++) {
        long r = zstd_decompress_wave(fp[s], (size_t)fl[s], inter + off, (size_t)cs[s], S, P);
        if (r < 0) return PGN_ERR_ZSTD_DECOMPRESS;
        dres[s] = (uint64_t)r;
        off += cs[s];
    }
    wave_sync();
    P.mark(0);
    uint64_t consumed = 0;
    const int bad = c5_merge_wave(inter, total, dres[1], dres[2], dres[3], out, n, &consumed);
    P.mark(6);
    if (bad) return PGN_ERR_CORRUPT;
    if (consumed != total) return PGN_ERR_REMAINING;
    return PGN_OK;
}

__global__ __launch_bounds__(64) void c5_decode_kernel(DecArgs a)
{
    const DecLayout lay = dec_layout();
    uint8_t* base = a.scratch + (size_t)blockIdx.x * a.slotBytes;
    DecScratch S;
    S.lit = base + lay.lit;
    S.seqs = (uint32_t*)(base + lay.seqs);
    S.maxSeq = kMaxDecSeq;
    S.tables = (z1::FseDTable*)(base + lay.tables);
    uint8_t* inter = base + lay.inter;
    PhaseProf P;
    P.init(a.prof);
    for (size_t c = blockIdx.x; c < a.nchunks; c += gridDim.x) {
        int st = c5_decode_chunk(a.in + a.inOffsets[c], a.inSizes[c], a.samples + a.sampleOffsets[c],
                                 a.sampleCounts[c], S, inter, P);
        if (lane_id() == 0) a.status[c] = st;
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

}  // namespace pgn

// =============================================================================================
// Host side: contexts, scratch, launches (C ABI)
// =============================================================================================
using namespace pgn;

struct pgn_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int numCUs = 0;
    size_t encSlotsMax = 0, decSlotsMax = 0;
    uint8_t* encScratch = nullptr;
    size_t encSlots = 0;
    uint32_t* epochs = nullptr;
    uint8_t* decScratch = nullptr;
    size_t decSlots = 0;
    // host-call staging (device buffers)
    uint8_t* stage = nullptr;
    size_t stageBytes = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t* prof = nullptr;  // [2][kPhases] phase cycles (encode, decode) when PGN_PHASE_PROFILE=1
    bool encTimed = false, decTimed = false;
    std::mutex mu;
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
    case PGN_ERR_UNSUPPORTED: return "Chunk larger than PGN_MAX_CHUNK_SAMPLES";
    case PGN_ERR_INVALID_ARG: return "Invalid argument";
    case PGN_ERR_HIP: return "HIP runtime error";
    case PGN_ERR_NO_DEVICE: return "No HIP device";
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
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&encPerCU, c5_encode_kernel, 64, 0));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&decPerCU, c5_decode_kernel, 64, 0));
    if (encPerCU < 1) encPerCU = 1;
    if (decPerCU < 1) decPerCU = 1;
    c->encSlotsMax = (size_t)c->numCUs * (size_t)(encPerCU > 16 ? 16 : encPerCU);
    c->decSlotsMax = (size_t)c->numCUs * (size_t)(decPerCU > 16 ? 16 : decPerCU);
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    const char* pe = getenv("PGN_PHASE_PROFILE");
    if (pe && pe[0] == '1') {
        HIPCHK(hipMalloc(&c->prof, 2 * kPhases * sizeof(uint64_t)));
        HIPCHK(hipMemset(c->prof, 0, 2 * kPhases * sizeof(uint64_t)));
        HIPCHK(hipDeviceSynchronize());
    }
    for (int i = 0; i < 4; i++) HIPCHK(hipEventCreate(&c->ev[i]));
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
    (void)hipFree(c->stage);
    (void)hipFree(c->prof);
    for (int i = 0; i < 4; i++) if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return PGN_OK;
}

void* pgn_ctx_stream(pgn_ctx* c) { return c ? (void*)c->stream : nullptr; }

static int ensure_enc(pgn_ctx* c, size_t slots)
{
    if (slots <= c->encSlots) return PGN_OK;
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->encScratch);
    (void)hipFree(c->epochs);
    c->encScratch = nullptr;
    c->epochs = nullptr;
    const size_t sb = enc_layout().bytes;
    HIPCHK(hipMalloc(&c->encScratch, sb * slots));
    HIPCHK(hipMalloc(&c->epochs, 4 * slots));
    // tag 0 never matches: a zeroed table is an empty table for every epoch >= 1.  The context
    // stream is non-blocking, so zero on it and wait before any launch (on any stream) uses it.
    HIPCHK(hipMemsetAsync(c->epochs, 0, 4 * slots, c->stream));
    HIPCHK(hipMemsetAsync(c->encScratch, 0, sb * slots, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->encSlots = slots;
    return PGN_OK;
}

static int ensure_dec(pgn_ctx* c, size_t slots)
{
    if (slots <= c->decSlots) return PGN_OK;
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->decScratch);
    c->decScratch = nullptr;
    HIPCHK(hipMalloc(&c->decScratch, dec_layout().bytes * slots));
    c->decSlots = slots;
    return PGN_OK;
}

static int launch_encode(pgn_ctx* c, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                         const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                         void* stream)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    size_t slots = nchunks < c->encSlotsMax ? nchunks : c->encSlotsMax;
    int rc = ensure_enc(c, slots);
    if (rc) return rc;
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
    a.scratch = c->encScratch;
    a.slotBytes = enc_layout().bytes;
    a.epochs = c->epochs;
    a.prof = c->prof;
    HIPCHK(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(c5_encode_kernel, dim3((unsigned)slots), dim3(64), 0, s, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[1], s));
    c->encTimed = true;
    return PGN_OK;
}

static int launch_decode(pgn_ctx* c, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                         const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                         const uint32_t* d_sample_counts, int32_t* d_status, void* stream)
{
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    size_t slots = nchunks < c->decSlotsMax ? nchunks : c->decSlotsMax;
    int rc = ensure_dec(c, slots);
    if (rc) return rc;
    DecArgs a;
    a.nchunks = nchunks;
    a.in = d_in;
    a.inOffsets = d_in_offsets;
    a.inSizes = d_in_sizes;
    a.samples = d_samples;
    a.sampleOffsets = d_sample_offsets;
    a.sampleCounts = d_sample_counts;
    a.status = d_status;
    a.scratch = c->decScratch;
    a.slotBytes = dec_layout().bytes;
    a.prof = c->prof ? c->prof + kPhases : nullptr;
    HIPCHK(hipEventRecord(c->ev[2], s));
    hipLaunchKernelGGL(c5_decode_kernel, dim3((unsigned)slots), dim3(64), 0, s, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[3], s));
    c->decTimed = true;
    return PGN_OK;
}

int pgn_compress_batch_device(pgn_ctx* c, size_t nchunks, const int16_t* d_samples, const uint64_t* d_sample_offsets,
                              const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
                              const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats,
                              void* stream)
{
    if (!c || !d_samples || !d_sample_offsets || !d_sample_counts || !d_out || !d_out_offsets || !d_out_caps ||
        !d_out_sizes || !d_status)
        return PGN_ERR_INVALID_ARG;
    if (nchunks == 0) return PGN_OK;
    std::lock_guard<std::mutex> g(c->mu);
    return launch_encode(c, nchunks, d_samples, d_sample_offsets, d_sample_counts, d_out, d_out_offsets, d_out_caps,
                         d_out_sizes, d_status, d_stats, stream);
}

int pgn_decompress_batch_device(pgn_ctx* c, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
                                const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets,
                                const uint32_t* d_sample_counts, int32_t* d_status, void* stream)
{
    if (!c || !d_in || !d_in_offsets || !d_in_sizes || !d_samples || !d_sample_offsets || !d_sample_counts || !d_status)
        return PGN_ERR_INVALID_ARG;
    if (nchunks == 0) return PGN_OK;
    std::lock_guard<std::mutex> g(c->mu);
    return launch_decode(c, nchunks, d_in, d_in_offsets, d_in_sizes, d_samples, d_sample_offsets, d_sample_counts,
                         d_status, stream);
}

int pgn_debug_phase_cycles(pgn_ctx* c, uint64_t* out, int n)
{
    if (!c || !out || n < 2 * kPhases) return PGN_ERR_INVALID_ARG;
    if (!c->prof) {
        memset(out, 0, sizeof(uint64_t) * 2 * kPhases);
        return PGN_OK;
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->prof, sizeof(uint64_t) * 2 * kPhases, hipMemcpyDeviceToHost));
    return PGN_OK;
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
    (void)hipFree(c->stage);
    c->stage = nullptr;
    size_t b = align_up(bytes, 1 << 20);
    HIPCHK(hipMalloc(&c->stage, b));
    c->stageBytes = b;
    return PGN_OK;
}

struct StageHdr {
    uint64_t off0, cnt0pad, outOff, outCap, outSize, inOff, inSize;
    uint32_t count;
    int32_t status;
    uint64_t stats[PGN_STATS_PER_CHUNK];
};

int pgn_compress_signal(pgn_ctx* c, const int16_t* samples, size_t n, uint8_t* dst, size_t cap, size_t* out_size)
{
    if (!c || (!samples && n) || !dst || !out_size) return PGN_ERR_INVALID_ARG;
    if (n > kMaxSamples) return PGN_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    const size_t hdrB = 256, inB = align_up(2 * n + 16, 256);
    int rc = ensure_stage(c, hdrB + inB + cap + 64);
    if (rc) return rc;
    uint8_t* dh = c->stage;
    uint8_t* din = c->stage + hdrB;
    uint8_t* dout = din + inB;
    StageHdr h{};
    h.off0 = 0;
    h.outOff = 0;
    h.outCap = cap;
    h.count = (uint32_t)n;
    HIPCHK(hipMemcpyAsync(dh, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    if (n) HIPCHK(hipMemcpyAsync(din, samples, 2 * n, hipMemcpyHostToDevice, c->stream));
    StageHdr* d = (StageHdr*)dh;
    rc = launch_encode(c, 1, (const int16_t*)din, &d->off0, &d->count, dout, &d->outOff, &d->outCap,
                                   &d->outSize, &d->status, d->stats, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(&h, dh, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *out_size = (size_t)h.outSize;
    if (h.status != PGN_OK) return h.status;
    HIPCHK(hipMemcpy(dst, dout, (size_t)h.outSize, hipMemcpyDeviceToHost));
    return PGN_OK;
}

int pgn_decompress_signal(pgn_ctx* c, const uint8_t* src, size_t len, int16_t* dst, size_t n)
{
    if (!c || (!src && len) || (!dst && n)) return PGN_ERR_INVALID_ARG;
    if (n > kMaxSamples) return PGN_ERR_UNSUPPORTED;
    const size_t hdrB = 256, inB = align_up(len + 16, 256);
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = ensure_stage(c, hdrB + inB + 2 * n + 64);
    if (rc) return rc;
    uint8_t* dh = c->stage;
    uint8_t* din = c->stage + hdrB;
    int16_t* dout = (int16_t*)(din + inB);
    StageHdr h{};
    h.inOff = 0;
    h.inSize = len;
    h.off0 = 0;
    h.count = (uint32_t)n;
    HIPCHK(hipMemcpyAsync(dh, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    if (len) HIPCHK(hipMemcpyAsync(din, src, len, hipMemcpyHostToDevice, c->stream));
    StageHdr* d = (StageHdr*)dh;
    rc = launch_decode(c, 1, din, &d->inOff, &d->inSize, dout, &d->off0, &d->count, &d->status,
                                         c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(&h, dh, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (h.status != PGN_OK) return h.status;
    if (n) HIPCHK(hipMemcpy(dst, dout, 2 * n, hipMemcpyDeviceToHost));
    return PGN_OK;
}

static pgn_ctx* g_default = nullptr;
static std::mutex g_default_mu;

int pgn_pinanoraw_compress_signal(const int16_t* signal, size_t signal_size, char* out, size_t* inout_size)
{
    if (!signal || !out || !inout_size) return PGN_ERR_INVALID_ARG;
    {
        std::lock_guard<std::mutex> g(g_default_mu);
        if (!g_default) {
            int rc = pgn_ctx_create(0, &g_default);
            if (rc) return rc;
        }
    }
    // pgnano::compress_signal allocates compressed_signal_max_size(n) (pgnano.cpp:66-68) ...
    const size_t cap = pgn_compressed_signal_max_size(signal_size);
    uint8_t* tmp = (uint8_t*)malloc(cap);
    if (!tmp) return PGN_ERR_INVALID_ARG;
    size_t sz = 0;
    int rc = pgn_compress_signal(g_default, signal, signal_size, tmp, cap, &sz);
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

}  // extern "C"
