// pgn_pod5.hip -- batched POD5 signal-table integration (include/pgnano_pod5.h): the reads of one
// pod5_add_reads_data call (c_api.cpp:1104-1129), chunked as the writer chunks them
// (file_writer.cpp:119-143), compressed by one batched launch and returned in the signal column
// layout; a reader's record batch of rows (signal_table_reader.cpp:294-318) decoded by one launch.
//
// Host memory in and out.  Per call: the samples (or blobs) are gathered into a pinned staging
// buffer and sent to HBM with one copy; the codec runs on the context's stream; the blobs, written at
// capacity-spaced offsets by the batch kernels, are packed on the device (an exclusive scan of the
// sizes, then one wave per chunk) so that only the compressed bytes cross PCIe on the way back.
#include <hip/hip_runtime.h>
#include <string.h>

#include <new>
#include <stdexcept>
#include <vector>

#include "../../include/pgnano_pod5.h"
#include "../../include/pgnano_pod5file.h"

namespace {

// exclusive scan of the sizes of the chunks that succeeded (a failed chunk counts 0: the multi-frame
// encoders report the reference's "Required size" there, which may exceed the chunk's capacity)
// -> offs[0..n], offs[n] = total; first[0] = index of the first non-OK status (n if none).  One
// workgroup of 1024 threads, tiles of 1024 with a running carry.
__global__ __launch_bounds__(1024) void pod5_scan_kernel(const uint64_t* sizes, const int32_t* status, uint64_t* offs,
                                                         uint32_t* first, uint32_t n)
{
    __shared__ uint64_t s[1024];
    __shared__ uint64_t carry;
    __shared__ uint32_t bad;
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        carry = 0;
        bad = n;
    }
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + t;
        const bool ok = i < n && status[i] == 0;
        const uint64_t v = ok ? sizes[i] : 0;
        if (i < n && !ok) atomicMin(&bad, i);
        s[t] = v;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
            const uint64_t a = t >= d ? s[t - d] : 0;
            __syncthreads();
            s[t] += a;
            __syncthreads();
        }
        if (i < n) offs[i] = carry + s[t] - v;
        __syncthreads();
        if (t == 1023) carry += s[1023];
        __syncthreads();
    }
    if (t == 0) {
        offs[n] = carry;
        first[0] = bad;
    }
}

// chunk g's blob: src + srcOff[g] -> dst + dstOff[g], size dstOff[g + 1] - dstOff[g]; one wave each
__global__ __launch_bounds__(64) void pod5_pack_kernel(const uint8_t* src, const uint64_t* srcOff, const uint64_t* dstOff,
                                                       uint8_t* dst, uint32_t n)
{
    const uint32_t g = blockIdx.x;
    if (g >= n) return;
    const uint8_t* a = src + srcOff[g];
    uint8_t* b = dst + dstOff[g];
    const uint64_t len = dstOff[g + 1] - dstOff[g];
    const uint32_t lane = threadIdx.x;
    // 16-byte pieces where both sides allow it, else bytes
    if ((((uintptr_t)a | (uintptr_t)b) & 15u) == 0) {
        uint64_t i = 16u * lane;
        for (; i + 16 <= len; i += 1024) *(uint4*)(b + i) = *(const uint4*)(a + i);
        for (uint64_t k = (len & ~(uint64_t)15) + lane; k < len; k += 64) b[k] = a[k];
    } else {
        for (uint64_t k = lane; k < len; k += 64) b[k] = a[k];
    }
}

thread_local char g_pod5_err[256];

}  // namespace

struct pgn_pod5_batch {
    pgn_ctx* ctx = nullptr;
    int codec = PGN_VARIANT_C5;
    uint32_t chunk = PGN_POD5_DEFAULT_CHUNK_SIZE;
    hipStream_t stream = nullptr;
    // pinned host staging, grown on demand
    uint8_t* hBuf = nullptr;
    size_t hBufCap = 0;
    // device buffers, grown on demand
    uint8_t* dBuf = nullptr;
    size_t dBufCap = 0;
    // results of the last call (what the out pointers refer to)
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> data;
    std::vector<uint32_t> samples, readIndex;
};

#define P5CHK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            snprintf(g_pod5_err, sizeof(g_pod5_err), "%s: %s", #x, hipGetErrorString(e_));        \
            return PGN_ERR_HIP;                                                                   \
        }                                                                                         \
    } while (0)

static size_t up256(size_t v) { return (v + 255) & ~(size_t)255; }

static int ensure_host(pgn_pod5_batch* b, size_t bytes)
{
    if (bytes <= b->hBufCap) return PGN_OK;
    if (b->hBuf) (void)hipHostFree(b->hBuf);
    b->hBuf = nullptr;
    const size_t cap = up256(bytes + bytes / 4);
    P5CHK(hipHostMalloc((void**)&b->hBuf, cap, hipHostMallocDefault));
    b->hBufCap = cap;
    return PGN_OK;
}

static int ensure_dev(pgn_pod5_batch* b, size_t bytes)
{
    if (bytes <= b->dBufCap) return PGN_OK;
    if (b->dBuf) {
        (void)hipStreamSynchronize(b->stream);
        (void)hipFree(b->dBuf);
    }
    b->dBuf = nullptr;
    const size_t cap = up256(bytes + bytes / 4);
    P5CHK(hipMalloc((void**)&b->dBuf, cap));
    b->dBufCap = cap;
    return PGN_OK;
}

// destination capacity of a chunk of n samples: pgnano max(2n + 26, 1024) (compressor.h:39-45),
// VBZ ZSTD_compressBound(svb16 max) (signal_compression.cpp:14-19)
static uint64_t chunk_cap(int codec, uint32_t n)
{
    return codec == PGN_POD5_CODEC_VBZ ? (uint64_t)pgn_vbz_compressed_signal_max_size(n)
                                       : (uint64_t)pgn_compressed_signal_max_size(n);
}

static int batch_compress(pgn_pod5_batch* b, size_t n, const int16_t* d_samples, const uint64_t* d_soff,
                          const uint32_t* d_cnt, uint8_t* d_out, const uint64_t* d_ooff, const uint64_t* d_caps,
                          uint64_t* d_sizes, int32_t* d_status)
{
    if (b->codec == PGN_POD5_CODEC_VBZ)
        return pgn_vbz_compress_batch_device(b->ctx, n, d_samples, d_soff, d_cnt, d_out, d_ooff, d_caps, d_sizes,
                                             d_status, nullptr, b->stream);
    return pgn_variant_compress_batch_device(b->ctx, b->codec, n, d_samples, d_soff, d_cnt, d_out, d_ooff, d_caps,
                                             d_sizes, d_status, nullptr, b->stream);
}

static int batch_decompress(pgn_pod5_batch* b, size_t n, const uint8_t* d_in, const uint64_t* d_ioff,
                            const uint64_t* d_isz, int16_t* d_samples, const uint64_t* d_soff, const uint32_t* d_cnt,
                            int32_t* d_status)
{
    if (b->codec == PGN_POD5_CODEC_VBZ)
        return pgn_vbz_decompress_batch_device(b->ctx, n, d_in, d_ioff, d_isz, d_samples, d_soff, d_cnt, d_status,
                                               b->stream);
    return pgn_variant_decompress_batch_device(b->ctx, b->codec, n, d_in, d_ioff, d_isz, d_samples, d_soff, d_cnt,
                                               d_status, b->stream);
}

extern "C" {

const char* pgn_pod5_last_error(void) { return g_pod5_err; }

int pgn_pod5_batch_create(pgn_ctx* ctx, int codec, uint32_t chunk_size, pgn_pod5_batch** out)
{
    if (!ctx || !out) return PGN_ERR_INVALID_ARG;
    if (codec != PGN_POD5_CODEC_VBZ && (codec < PGN_VARIANT_C5 || codec > PGN_VARIANT_VBZ0)) return PGN_ERR_INVALID_ARG;
    if (chunk_size == 0) chunk_size = PGN_POD5_DEFAULT_CHUNK_SIZE;
    if (chunk_size > PGN_MAX_CHUNK_SAMPLES) return PGN_ERR_UNSUPPORTED;
    pgn_pod5_batch* b = new pgn_pod5_batch();
    b->ctx = ctx;
    b->codec = codec;
    b->chunk = chunk_size;
    b->stream = (hipStream_t)pgn_ctx_stream(ctx);
    *out = b;
    return PGN_OK;
}

int pgn_pod5_batch_destroy(pgn_pod5_batch* b)
{
    if (!b) return PGN_ERR_INVALID_ARG;
    (void)hipStreamSynchronize(b->stream);
    if (b->dBuf) (void)hipFree(b->dBuf);
    if (b->hBuf) (void)hipHostFree(b->hBuf);
    delete b;
    return PGN_OK;
}

int pgn_pod5_compress_reads(pgn_pod5_batch* b, uint32_t read_count, const int16_t* const* signal,
                            const uint32_t* signal_size, size_t* out_chunk_count, const uint64_t** out_offsets,
                            const uint8_t** out_data, const uint32_t** out_samples, const uint32_t** out_read_index)
{
    if (!b || (read_count && (!signal || !signal_size)) || !out_chunk_count || !out_offsets || !out_data ||
        !out_samples || !out_read_index)
        return PGN_ERR_INVALID_ARG;
    // the writer's chunking (file_writer.cpp:119-143): chunk k of a read = samples [k*cs, min((k+1)*cs, n))
    b->samples.clear();
    b->readIndex.clear();
    size_t total = 0;
    for (uint32_t r = 0; r < read_count; r++) {
        if (signal_size[r] && !signal[r]) return PGN_ERR_INVALID_ARG;
        for (uint32_t s = 0; s < signal_size[r]; s += b->chunk) {
            b->samples.push_back(signal_size[r] - s < b->chunk ? signal_size[r] - s : b->chunk);
            b->readIndex.push_back(r);
        }
        total += signal_size[r];
    }
    const size_t n = b->samples.size();
    *out_chunk_count = 0;
    b->offsets.assign(n + 1, 0);
    b->data.clear();
    if (n == 0) {
        *out_offsets = b->offsets.data();
        *out_data = b->data.data();
        *out_samples = b->samples.data();
        *out_read_index = b->readIndex.data();
        return PGN_OK;
    }
    // device layout: samples | sample offsets | counts | blob offsets | caps | sizes | status |
    //                packed offsets (n + 1) | first bad | blobs (capacity-spaced) | packed blobs
    uint64_t capTotal = 0;
    for (size_t i = 0; i < n; i++) capTotal += chunk_cap(b->codec, b->samples[i]);
    const size_t oSamples = 0, oSoff = up256(2 * total), oCnt = oSoff + up256(8 * n), oOoff = oCnt + up256(4 * n),
                 oCaps = oOoff + up256(8 * n), oSizes = oCaps + up256(8 * n), oStatus = oSizes + up256(8 * n),
                 oPoff = oStatus + up256(4 * n), oFirst = oPoff + up256(8 * (n + 1)), oBlobs = oFirst + 256,
                 oPacked = oBlobs + up256(capTotal), devBytes = oPacked + up256(capTotal);
    int rc = ensure_dev(b, devBytes);
    if (rc) return rc;
    // host staging: samples in, packed blobs out (the same region) | per-chunk arrays | offsets back
    const size_t hostMeta = up256(8 * n) * 3 + up256(4 * n);
    const size_t hBase = up256(2 * total > capTotal ? 2 * total : capTotal);
    rc = ensure_host(b, hBase + hostMeta + up256(8 * (n + 1)) + 256);
    if (rc) return rc;
    // stage: the samples in read order (chunks of a read are contiguous), then the per-chunk arrays
    uint8_t* h = b->hBuf;
    size_t at = 0;
    for (uint32_t r = 0; r < read_count; r++) {
        if (signal_size[r]) memcpy(h + at, signal[r], 2 * (size_t)signal_size[r]);
        at += 2 * (size_t)signal_size[r];
    }
    uint64_t* hSoff = (uint64_t*)(h + hBase);
    uint32_t* hCnt = (uint32_t*)((uint8_t*)hSoff + up256(8 * n));
    uint64_t* hOoff = (uint64_t*)((uint8_t*)hCnt + up256(4 * n));
    uint64_t* hCaps = (uint64_t*)((uint8_t*)hOoff + up256(8 * n));
    uint64_t so = 0, oo = 0;
    for (size_t i = 0; i < n; i++) {
        hSoff[i] = so;
        hCnt[i] = b->samples[i];
        hOoff[i] = oo;
        hCaps[i] = chunk_cap(b->codec, b->samples[i]);
        so += b->samples[i];
        oo += hCaps[i];
    }
    uint8_t* d = b->dBuf;
    P5CHK(hipMemcpyAsync(d + oSamples, h, 2 * total, hipMemcpyHostToDevice, b->stream));
    P5CHK(hipMemcpyAsync(d + oSoff, hSoff, (uint8_t*)hCaps + 8 * n - (uint8_t*)hSoff, hipMemcpyHostToDevice, b->stream));
    rc = batch_compress(b, n, (const int16_t*)(d + oSamples), (const uint64_t*)(d + oSoff), (const uint32_t*)(d + oCnt),
                        d + oBlobs, (const uint64_t*)(d + oOoff), (const uint64_t*)(d + oCaps), (uint64_t*)(d + oSizes),
                        (int32_t*)(d + oStatus));
    if (rc) return rc;
    hipLaunchKernelGGL(pod5_scan_kernel, dim3(1), dim3(1024), 0, b->stream, (const uint64_t*)(d + oSizes),
                       (const int32_t*)(d + oStatus), (uint64_t*)(d + oPoff), (uint32_t*)(d + oFirst), (uint32_t)n);
    hipLaunchKernelGGL(pod5_pack_kernel, dim3((unsigned)n), dim3(64), 0, b->stream, (const uint8_t*)(d + oBlobs),
                       (const uint64_t*)(d + oOoff), (const uint64_t*)(d + oPoff), d + oPacked, (uint32_t)n);
    P5CHK(hipGetLastError());
    // offsets + first failing chunk back, then exactly the packed bytes
    uint64_t* hPoff = (uint64_t*)(h + hBase + hostMeta);
    uint32_t* hFirst = (uint32_t*)((uint8_t*)hPoff + up256(8 * (n + 1)));
    P5CHK(hipMemcpyAsync(hPoff, d + oPoff, 8 * (n + 1), hipMemcpyDeviceToHost, b->stream));
    P5CHK(hipMemcpyAsync(hFirst, d + oFirst, 4, hipMemcpyDeviceToHost, b->stream));
    P5CHK(hipStreamSynchronize(b->stream));
    if (*hFirst < n) {
        int32_t s = 0;
        P5CHK(hipMemcpy(&s, d + oStatus + 4 * (size_t)*hFirst, 4, hipMemcpyDeviceToHost));
        *out_chunk_count = *hFirst;
        return s ? s : PGN_ERR_INVALID_ARG;
    }
    memcpy(b->offsets.data(), hPoff, 8 * (n + 1));
    const uint64_t packed = b->offsets[n];
    P5CHK(hipMemcpyAsync(h, d + oPacked, packed, hipMemcpyDeviceToHost, b->stream));
    P5CHK(hipStreamSynchronize(b->stream));
    b->data.assign(h, h + packed);
    *out_chunk_count = n;
    *out_offsets = b->offsets.data();
    *out_data = b->data.data();
    *out_samples = b->samples.data();
    *out_read_index = b->readIndex.data();
    return PGN_OK;
}

int pgn_pod5_decompress_rows(pgn_pod5_batch* b, uint32_t row_count, const uint64_t* offsets, const uint8_t* data,
                             const uint32_t* samples, int16_t* out, int32_t* row_status)
{
    if (!b || (row_count && (!offsets || !samples))) return PGN_ERR_INVALID_ARG;
    if (row_count == 0) return PGN_OK;
    const size_t n = row_count;
    const uint64_t bytes = offsets[n] - offsets[0];
    if (offsets[n] < offsets[0] || (bytes && !data)) return PGN_ERR_INVALID_ARG;
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) {
        if (offsets[i + 1] < offsets[i]) return PGN_ERR_INVALID_ARG;
        total += samples[i];
    }
    if (total && !out) return PGN_ERR_INVALID_ARG;
    // device: blobs | blob offsets | blob sizes | sample offsets | counts | status | samples
    const size_t oIn = 0, oIoff = up256(bytes), oIsz = oIoff + up256(8 * n), oSoff = oIsz + up256(8 * n),
                 oCnt = oSoff + up256(8 * n), oStatus = oCnt + up256(4 * n), oOut = oStatus + up256(4 * n),
                 devBytes = oOut + up256(2 * total);
    int rc = ensure_dev(b, devBytes);
    if (rc) return rc;
    const size_t metaBytes = up256(8 * n) * 3 + up256(4 * n);
    rc = ensure_host(b, (bytes > 2 * total ? bytes : 2 * total) + metaBytes + up256(4 * n));
    if (rc) return rc;
    uint8_t* h = b->hBuf;
    if (bytes) memcpy(h, data + offsets[0], bytes);
    uint64_t* hIoff = (uint64_t*)(h + up256(bytes > 2 * total ? bytes : 2 * total));
    uint64_t* hIsz = (uint64_t*)((uint8_t*)hIoff + up256(8 * n));
    uint64_t* hSoff = (uint64_t*)((uint8_t*)hIsz + up256(8 * n));
    uint32_t* hCnt = (uint32_t*)((uint8_t*)hSoff + up256(8 * n));
    int32_t* hStatus = (int32_t*)((uint8_t*)hCnt + up256(4 * n));
    uint64_t so = 0;
    for (size_t i = 0; i < n; i++) {
        hIoff[i] = offsets[i] - offsets[0];
        hIsz[i] = offsets[i + 1] - offsets[i];
        hSoff[i] = so;
        hCnt[i] = samples[i];
        so += samples[i];
    }
    uint8_t* d = b->dBuf;
    if (bytes) P5CHK(hipMemcpyAsync(d + oIn, h, bytes, hipMemcpyHostToDevice, b->stream));
    P5CHK(hipMemcpyAsync(d + oIoff, hIoff, (uint8_t*)hCnt + 4 * n - (uint8_t*)hIoff, hipMemcpyHostToDevice, b->stream));
    rc = batch_decompress(b, n, d + oIn, (const uint64_t*)(d + oIoff), (const uint64_t*)(d + oIsz),
                          (int16_t*)(d + oOut), (const uint64_t*)(d + oSoff), (const uint32_t*)(d + oCnt),
                          (int32_t*)(d + oStatus));
    if (rc) return rc;
    P5CHK(hipMemcpyAsync(hStatus, d + oStatus, 4 * n, hipMemcpyDeviceToHost, b->stream));
    if (total) P5CHK(hipMemcpyAsync(h, d + oOut, 2 * total, hipMemcpyDeviceToHost, b->stream));
    P5CHK(hipStreamSynchronize(b->stream));
    if (total) memcpy(out, h, 2 * total);
    int first = PGN_OK;
    for (size_t i = 0; i < n; i++) {
        if (row_status) row_status[i] = hStatus[i];
        if (first == PGN_OK && hStatus[i] != PGN_OK) first = hStatus[i];
    }
    return first;
}

// pgnano_pod5file.h: `copy --pgnano | --VBZ` of a file's signal table.  Device-resident between the
// two launches: blobs up -> batched decode into one sample buffer -> batched encode -> device-side
// pack -> packed blobs down.
static int transcode_impl(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                          int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats);

// the host vectors are sized from the file: an allocation failure (or any exception) becomes a
// status instead of crossing the C ABI
int pgn_pod5_transcode_file(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                            int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats)
{
    try {
        return transcode_impl(ctx, in_path, out_path, dst_signal_type, pgnano_variant, rows_per_batch, stats);
    } catch (const std::bad_alloc&) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "out of host memory");
        return PGN_ERR_IO;
    } catch (const std::exception& e) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", e.what());
        return PGN_ERR_CORRUPT;
    }
}

}  // extern "C"

static int transcode_impl(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                          int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats)
{
    if (!ctx || !in_path || !out_path || dst_signal_type < PGN_POD5_SIGNAL_UNCOMPRESSED ||
        dst_signal_type > PGN_POD5_SIGNAL_PGNANO || pgnano_variant < PGN_VARIANT_C5 || pgnano_variant > PGN_VARIANT_VBZ0)
        return PGN_ERR_INVALID_ARG;
    pgn_pod5_file* f = nullptr;
    int rc = pgn_pod5_file_open(in_path, &f);
    if (rc) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", pgn_pod5_file_error());
        return rc;
    }
    uint64_t rows = 0, dataBytes = 0, total = 0;
    uint32_t nb = 0;
    int srcType = 0;
    pgn_pod5_signal_info(f, &rows, &nb, &srcType, &dataBytes, &total);
    std::vector<uint8_t> ids(16 * rows), data(dataBytes), outData;
    std::vector<uint32_t> samples(rows);
    std::vector<uint64_t> offs(rows + 1), outOffs(rows + 1, 0);
    pgn_pod5_signal_read(f, ids.data(), samples.data(), offs.data(), data.data());
    const int srcCodec = srcType == PGN_POD5_SIGNAL_VBZ ? PGN_POD5_CODEC_VBZ : pgnano_variant;
    const int dstCodec = dst_signal_type == PGN_POD5_SIGNAL_VBZ ? PGN_POD5_CODEC_VBZ : pgnano_variant;
    const size_t n = (size_t)rows;
    float decMs = 0, encMs = 0;
    uint8_t* d = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    const hipStream_t stream = (hipStream_t)pgn_ctx_stream(ctx);
    pgn_pod5_batch src, dst;
    src.ctx = dst.ctx = ctx;
    src.stream = dst.stream = stream;
    src.codec = srcCodec;
    dst.codec = dstCodec;
    auto body = [&]() -> int {
        if (n >= (1u << 31)) return PGN_ERR_UNSUPPORTED;
        for (size_t i = 0; i < n; i++)
            if (samples[i] > PGN_MAX_CHUNK_SAMPLES) {
                snprintf(g_pod5_err, sizeof(g_pod5_err), "row %zu: %u samples above PGN_MAX_CHUNK_SAMPLES", i,
                         samples[i]);
                return PGN_ERR_UNSUPPORTED;
            }
        if (n == 0) return PGN_OK;
        uint64_t capTotal = 0;
        for (size_t i = 0; i < n; i++) capTotal += chunk_cap(dstCodec, samples[i]);
        // device: samples | sample offsets | counts | status | blobs in | in offsets | in sizes |
        //         blobs out (capacity-spaced) | out offsets | caps | sizes | packed offsets | first | packed
        const size_t oSamples = 0, oSoff = up256(2 * total), oCnt = oSoff + up256(8 * n), oStatus = oCnt + up256(4 * n),
                     oIn = oStatus + up256(4 * n), oIoff = oIn + up256(dataBytes), oIsz = oIoff + up256(8 * n),
                     oOut = oIsz + up256(8 * n), oOoff = oOut + up256(capTotal), oCaps = oOoff + up256(8 * n),
                     oSizes = oCaps + up256(8 * n), oPoff = oSizes + up256(8 * n), oFirst = oPoff + up256(8 * (n + 1)),
                     oPacked = oFirst + 256, devBytes = oPacked + up256(capTotal);
        P5CHK(hipMalloc((void**)&d, devBytes));
        for (auto& e : ev) P5CHK(hipEventCreate(&e));
        // per-row arrays, staged in one host block
        std::vector<uint64_t> meta(6 * n + 1);
        uint64_t *hSoff = meta.data(), *hIoff = hSoff + n, *hIsz = hIoff + n, *hOoff = hIsz + n, *hCaps = hOoff + n;
        uint32_t* hCnt = (uint32_t*)(hCaps + n);
        uint64_t so = 0, oo = 0;
        for (size_t i = 0; i < n; i++) {
            hSoff[i] = so;
            so += samples[i];
            hIoff[i] = offs[i];
            hIsz[i] = offs[i + 1] - offs[i];
            hCaps[i] = chunk_cap(dstCodec, samples[i]);
            hOoff[i] = oo;
            oo += hCaps[i];
            hCnt[i] = samples[i];
        }
        P5CHK(hipMemcpyAsync(d + oSoff, hSoff, 8 * n, hipMemcpyHostToDevice, stream));
        P5CHK(hipMemcpyAsync(d + oCnt, hCnt, 4 * n, hipMemcpyHostToDevice, stream));
        P5CHK(hipMemcpyAsync(d + oOoff, hOoff, 8 * n, hipMemcpyHostToDevice, stream));
        P5CHK(hipMemcpyAsync(d + oCaps, hCaps, 8 * n, hipMemcpyHostToDevice, stream));
        if (srcType == PGN_POD5_SIGNAL_UNCOMPRESSED) {
            for (size_t i = 0; i < n; i++)
                if (hIsz[i] != 2ull * samples[i]) return PGN_ERR_CORRUPT;
            if (dataBytes) P5CHK(hipMemcpyAsync(d + oSamples, data.data(), dataBytes, hipMemcpyHostToDevice, stream));
        } else {
            if (dataBytes) P5CHK(hipMemcpyAsync(d + oIn, data.data(), dataBytes, hipMemcpyHostToDevice, stream));
            P5CHK(hipMemcpyAsync(d + oIoff, hIoff, 8 * n, hipMemcpyHostToDevice, stream));
            P5CHK(hipMemcpyAsync(d + oIsz, hIsz, 8 * n, hipMemcpyHostToDevice, stream));
            P5CHK(hipEventRecord(ev[0], stream));
            int r = batch_decompress(&src, n, d + oIn, (const uint64_t*)(d + oIoff), (const uint64_t*)(d + oIsz),
                                     (int16_t*)(d + oSamples), (const uint64_t*)(d + oSoff),
                                     (const uint32_t*)(d + oCnt), (int32_t*)(d + oStatus));
            if (r) return r;
            P5CHK(hipEventRecord(ev[1], stream));
            std::vector<int32_t> st(n);
            P5CHK(hipMemcpyAsync(st.data(), d + oStatus, 4 * n, hipMemcpyDeviceToHost, stream));
            P5CHK(hipStreamSynchronize(stream));
            P5CHK(hipEventElapsedTime(&decMs, ev[0], ev[1]));
            for (size_t i = 0; i < n; i++)
                if (st[i] != PGN_OK) {
                    snprintf(g_pod5_err, sizeof(g_pod5_err), "row %zu: decode status %d", i, st[i]);
                    return st[i];
                }
        }
        if (dst_signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED) {
            outData.resize(2 * total);
            if (total) P5CHK(hipMemcpyAsync(outData.data(), d + oSamples, 2 * total, hipMemcpyDeviceToHost, stream));
            P5CHK(hipStreamSynchronize(stream));
            for (size_t i = 0; i < n; i++) outOffs[i + 1] = outOffs[i] + 2ull * samples[i];
            return PGN_OK;
        }
        P5CHK(hipEventRecord(ev[2], stream));
        int r = batch_compress(&dst, n, (const int16_t*)(d + oSamples), (const uint64_t*)(d + oSoff),
                               (const uint32_t*)(d + oCnt), d + oOut, (const uint64_t*)(d + oOoff),
                               (const uint64_t*)(d + oCaps), (uint64_t*)(d + oSizes), (int32_t*)(d + oStatus));
        if (r) return r;
        P5CHK(hipEventRecord(ev[3], stream));
        hipLaunchKernelGGL(pod5_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint64_t*)(d + oSizes),
                           (const int32_t*)(d + oStatus), (uint64_t*)(d + oPoff), (uint32_t*)(d + oFirst), (uint32_t)n);
        hipLaunchKernelGGL(pod5_pack_kernel, dim3((unsigned)n), dim3(64), 0, stream, (const uint8_t*)(d + oOut),
                           (const uint64_t*)(d + oOoff), (const uint64_t*)(d + oPoff), d + oPacked, (uint32_t)n);
        P5CHK(hipGetLastError());
        uint32_t first = 0;
        P5CHK(hipMemcpyAsync(outOffs.data(), d + oPoff, 8 * (n + 1), hipMemcpyDeviceToHost, stream));
        P5CHK(hipMemcpyAsync(&first, d + oFirst, 4, hipMemcpyDeviceToHost, stream));
        P5CHK(hipStreamSynchronize(stream));
        P5CHK(hipEventElapsedTime(&encMs, ev[2], ev[3]));
        if (first < n) {
            int32_t s = 0;
            P5CHK(hipMemcpy(&s, d + oStatus + 4 * (size_t)first, 4, hipMemcpyDeviceToHost));
            snprintf(g_pod5_err, sizeof(g_pod5_err), "row %u: encode status %d", first, s);
            return s ? s : PGN_ERR_INVALID_ARG;
        }
        outData.resize(outOffs[n]);
        if (outOffs[n]) P5CHK(hipMemcpyAsync(outData.data(), d + oPacked, outOffs[n], hipMemcpyDeviceToHost, stream));
        P5CHK(hipStreamSynchronize(stream));
        return PGN_OK;
    };
    rc = body();
    if (d) {
        (void)hipStreamSynchronize(stream);
        (void)hipFree(d);
    }
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    if (rc == PGN_OK)
    {
        rc = pgn_pod5_write_file(out_path, f, dst_signal_type, rows, ids.data(), samples.data(), outOffs.data(),
                                 outData.data(), rows_per_batch, nullptr, nullptr);
        if (rc) snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", pgn_pod5_file_error());
    }
    if (rc == PGN_OK && stats) {
        stats->rows = rows;
        stats->samples = total;
        stats->in_bytes = dataBytes;
        stats->out_bytes = outOffs[n];
        stats->decode_ms = decMs;
        stats->encode_ms = encMs;
    }
    pgn_pod5_file_close(f);
    return rc;
}


