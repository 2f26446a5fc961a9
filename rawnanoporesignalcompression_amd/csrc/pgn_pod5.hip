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

#include <condition_variable>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <stdexcept>
#include <vector>

#include "../../include/pgnano_pod5.h"
#include "../../include/pgnano_pod5file.h"
#include "pgn_internal.h"

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

// ---------------------------------------------------------------------------------------------
// Host copy workers: the pageable <-> pinned copies of the batch calls are split over a few
// persistent threads (one thread moves ~5-10 GB/s; the batch calls need 20+ GB/s to keep up with
// PCIe and the codec).  PGN_HOST_THREADS overrides the count (default min(8, hardware threads)).
// ---------------------------------------------------------------------------------------------
struct CopyJob {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};

class CopyPool {
public:
    explicit CopyPool(int nthreads)
    {
        for (int t = 1; t < nthreads; t++) th_.emplace_back([this, t] { worker(t); });
        n_ = nthreads;
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // all jobs, byte-balanced over the workers and the calling thread
    void run(const CopyJob* jobs, size_t njobs)
    {
        size_t total = 0;
        for (size_t i = 0; i < njobs; i++) total += jobs[i].n;
        if (total == 0) return;
        if (n_ == 1 || total < (1u << 20)) {
            for (size_t i = 0; i < njobs; i++) memcpy(jobs[i].dst, jobs[i].src, jobs[i].n);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            jobs_ = jobs;
            njobs_ = njobs;
            total_ = total;
            pending_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        share(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

private:
    // thread t copies bytes [t * total / n, (t + 1) * total / n) of the concatenated jobs
    void share(int t)
    {
        const size_t a = total_ * (size_t)t / (size_t)n_, b = total_ * (size_t)(t + 1) / (size_t)n_;
        size_t base = 0;
        for (size_t i = 0; i < njobs_ && base < b; i++) {
            const size_t lo = base, hi = base + jobs_[i].n;
            base = hi;
            if (hi <= a) continue;
            const size_t x = lo < a ? a - lo : 0, y = (hi < b ? hi : b) - lo;
            memcpy(jobs_[i].dst + x, jobs_[i].src + x, y - x);
        }
    }
    void worker(int t)
    {
        uint64_t seen = 0;
        while (true) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            share(t);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    int n_ = 1;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const CopyJob* jobs_ = nullptr;
    size_t njobs_ = 0, total_ = 0;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

static int host_threads()
{
    if (const char* v = getenv("PGN_HOST_THREADS")) {
        const int x = atoi(v);
        if (x > 0) return x > 64 ? 64 : x;
    }
    const unsigned h = std::thread::hardware_concurrency();
    return h == 0 ? 4 : (h < 8 ? (int)h : 8);
}

// sub-batch size of the pipelined calls (PGN_POD5_SUBBATCH_MB, default 64 MiB of input: measured best
// of 16 / 32 / 64 MiB with 4 / 8 / 16 copy threads, 9-11 GS/s each way on 1,000 x 100,000-sample reads)
static size_t sub_batch_bytes()
{
    if (const char* v = getenv("PGN_POD5_SUBBATCH_MB")) {
        const long x = atol(v);
        if (x > 0) return (size_t)x << 20;
    }
    return (size_t)64 << 20;
}

// A pinned host or device buffer that grows on demand (contents are not kept across growth).
struct PinBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
};
struct DevBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
};

struct pgn_pod5_batch {
    pgn_ctx* ctx = nullptr;
    int codec = PGN_VARIANT_C5;
    uint32_t chunk = PGN_POD5_DEFAULT_CHUNK_SIZE;
    hipStream_t stream = nullptr;  // the context's stream: codec launches, scan and pack
    hipStream_t copy = nullptr;    // host <-> device transfers
    CopyPool* pool = nullptr;
    // two pipeline slots: pinned staging and device buffers of one sub-batch each
    PinBuf hIn[2], hMeta[2], hRes[2];
    DevBuf dIn[2], dMeta[2], dOut[2], dPacked[2];
    hipEvent_t evH2D[2] = {nullptr, nullptr}, evComp[2] = {nullptr, nullptr}, evD2H[2] = {nullptr, nullptr};
    PinBuf hAll;  // compress: every packed blob of the call (what *out_data points to)
    // results of the last call (what the out pointers refer to)
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> samples, readIndex;
    std::vector<uint64_t> readStart;  // compress: first sample of each chunk within its read
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

// grow a pinned / device buffer (the caller has made sure no queued work still uses it)
static int ensure_pin(PinBuf& b, size_t bytes)
{
    if (bytes <= b.cap) return PGN_OK;
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t cap = up256(bytes + bytes / 4);
    P5CHK(hipHostMalloc((void**)&b.p, cap, hipHostMallocDefault));
    b.cap = cap;
    return PGN_OK;
}
static int ensure_devbuf(DevBuf& b, size_t bytes)
{
    if (bytes <= b.cap) return PGN_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t cap = up256(bytes + bytes / 4);
    P5CHK(hipMalloc((void**)&b.p, cap));
    b.cap = cap;
    return PGN_OK;
}

// destination capacity of a chunk of n samples: pgnano max(2n + 26, 1024) (compressor.h:39-45),
// VBZ ZSTD_compressBound(svb16 max) (signal_compression.cpp:14-19)
static uint64_t chunk_cap(int codec, uint32_t n)
{
    return codec == PGN_POD5_CODEC_VBZ ? (uint64_t)pgn_vbz_compressed_signal_max_size(n)
                                       : (uint64_t)pgn_compressed_signal_max_size(n);
}

// maxN: the largest sample count of the call's chunks (known on the host here: no large-chunk scan
// unless a chunk needs the large pass)
static int batch_compress(pgn_pod5_batch* b, size_t n, const int16_t* d_samples, const uint64_t* d_soff,
                          const uint32_t* d_cnt, uint8_t* d_out, const uint64_t* d_ooff, const uint64_t* d_caps,
                          uint64_t* d_sizes, int32_t* d_status, uint32_t maxN)
{
    return pgn_compress_batch_bounded(b->ctx, b->codec, maxN ? maxN : 1u, n, d_samples, d_soff, d_cnt, d_out, d_ooff,
                                      d_caps, d_sizes, d_status, nullptr, b->stream);
}

static int batch_decompress(pgn_pod5_batch* b, size_t n, const uint8_t* d_in, const uint64_t* d_ioff,
                            const uint64_t* d_isz, int16_t* d_samples, const uint64_t* d_soff, const uint32_t* d_cnt,
                            int32_t* d_status, uint32_t maxN)
{
    return pgn_decompress_batch_bounded(b->ctx, b->codec, maxN ? maxN : 1u, n, d_in, d_ioff, d_isz, d_samples, d_soff,
                                        d_cnt, d_status, b->stream);
}

// every queued transfer and launch of the batch has finished
static void batch_drain(pgn_pod5_batch* b)
{
    (void)hipStreamSynchronize(b->copy);
    (void)hipStreamSynchronize(b->stream);
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
    P5CHK(hipStreamCreateWithFlags(&b->copy, hipStreamNonBlocking));
    for (int s = 0; s < 2; s++) {
        P5CHK(hipEventCreateWithFlags(&b->evH2D[s], hipEventDisableTiming));
        P5CHK(hipEventCreateWithFlags(&b->evComp[s], hipEventDisableTiming));
        P5CHK(hipEventCreateWithFlags(&b->evD2H[s], hipEventDisableTiming));
    }
    b->pool = new CopyPool(host_threads());
    *out = b;
    return PGN_OK;
}

int pgn_pod5_batch_destroy(pgn_pod5_batch* b)
{
    if (!b) return PGN_ERR_INVALID_ARG;
    batch_drain(b);
    for (int s = 0; s < 2; s++) {
        for (PinBuf* h : {&b->hIn[s], &b->hMeta[s], &b->hRes[s]})
            if (h->p) (void)hipHostFree(h->p);
        for (DevBuf* d : {&b->dIn[s], &b->dMeta[s], &b->dOut[s], &b->dPacked[s]})
            if (d->p) (void)hipFree(d->p);
        for (hipEvent_t e : {b->evH2D[s], b->evComp[s], b->evD2H[s]})
            if (e) (void)hipEventDestroy(e);
    }
    if (b->hAll.p) (void)hipHostFree(b->hAll.p);
    if (b->copy) (void)hipStreamDestroy(b->copy);
    delete b->pool;
    delete b;
    return PGN_OK;
}

// Sub-batches of whole chunks (compress) or rows (decompress), about sub_batch_bytes() of input each.
static void split_subs(const std::vector<uint64_t>& bytesPer, size_t n, std::vector<size_t>& bounds)
{
    const size_t target = sub_batch_bytes();
    bounds.assign(1, 0);
    size_t acc = 0;
    for (size_t i = 0; i < n; i++) {
        if (acc > 0 && acc + bytesPer[i] > target) {
            bounds.push_back(i);
            acc = 0;
        }
        acc += bytesPer[i];
    }
    bounds.push_back(n);
}

// Compress pipeline over sub-batches j (chunks [c0, c1)), two slots s = j % 2:
//   host   : the sub-batch's samples -> hIn[s] (copy workers), its per-chunk arrays -> hMeta[s];
//   copy   : hIn/hMeta -> dIn/dMeta (after the compute of j - 2 has read them);
//   stream : codec + scan + pack into dPacked[s] (after the download of j - 2 has read it), packed
//            offsets and the first failing chunk -> hRes[s];
//   then, one sub-batch behind: the host reads hRes and the copy stream downloads the packed blobs
//   straight into the call's output (hAll), so that the packed bytes cross PCIe once and need no
//   further host copy.
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
    b->readStart.clear();
    for (uint32_t r = 0; r < read_count; r++) {
        if (signal_size[r] && !signal[r]) return PGN_ERR_INVALID_ARG;
        for (uint32_t s = 0; s < signal_size[r]; s += b->chunk) {
            b->samples.push_back(signal_size[r] - s < b->chunk ? signal_size[r] - s : b->chunk);
            b->readIndex.push_back(r);
            b->readStart.push_back(s);
        }
    }
    const size_t n = b->samples.size();
    *out_chunk_count = 0;
    b->offsets.assign(n + 1, 0);
    *out_offsets = b->offsets.data();
    *out_samples = b->samples.data();
    *out_read_index = b->readIndex.data();
    *out_data = b->hAll.p;
    if (n == 0) return PGN_OK;
    std::vector<uint64_t> caps(n), inBytes(n);
    uint64_t capAll = 0;
    for (size_t i = 0; i < n; i++) {
        caps[i] = chunk_cap(b->codec, b->samples[i]);
        inBytes[i] = 2ull * b->samples[i];
        capAll += caps[i];
    }
    std::vector<size_t> sb;
    split_subs(inBytes, n, sb);
    const size_t nsub = sb.size() - 1;
    // slot sizes: the largest sub-batch
    size_t maxIn = 0, maxCap = 0, maxN = 0;
    for (size_t j = 0; j < nsub; j++) {
        uint64_t a = 0, c = 0;
        for (size_t i = sb[j]; i < sb[j + 1]; i++) {
            a += inBytes[i];
            c += caps[i];
        }
        maxIn = a > maxIn ? a : maxIn;
        maxCap = c > maxCap ? c : maxCap;
        maxN = sb[j + 1] - sb[j] > maxN ? sb[j + 1] - sb[j] : maxN;
    }
    // per-slot metadata: soff | cnt | ooff | caps (uploaded), sizes | status | poff | first (device)
    const size_t mSoff = 0, mCnt = up256(8 * maxN), mOoff = mCnt + up256(4 * maxN), mCaps = mOoff + up256(8 * maxN),
                 mUp = mCaps + up256(8 * maxN), mSizes = mUp, mStatus = mSizes + up256(8 * maxN),
                 mPoff = mStatus + up256(4 * maxN), mFirst = mPoff + up256(8 * (maxN + 1)), mAll = mFirst + 256;
    batch_drain(b);  // buffers may grow below
    int rc = ensure_pin(b->hAll, capAll);
    if (rc) return rc;
    *out_data = b->hAll.p;
    for (int s = 0; s < 2 && s < (int)nsub; s++) {
        if ((rc = ensure_pin(b->hIn[s], maxIn)) || (rc = ensure_pin(b->hMeta[s], mUp)) ||
            (rc = ensure_pin(b->hRes[s], up256(8 * (maxN + 1)) + 256)) || (rc = ensure_devbuf(b->dIn[s], maxIn)) ||
            (rc = ensure_devbuf(b->dMeta[s], mAll)) || (rc = ensure_devbuf(b->dOut[s], maxCap)) ||
            (rc = ensure_devbuf(b->dPacked[s], maxCap)))
            return rc;
    }
    // read r's samples in this sub-batch: the chunks of a read are consecutive, so one copy per read run
    std::vector<CopyJob> jobs;
    uint64_t outBase = 0;
    int err = PGN_OK;
    size_t errChunk = n;
    auto finish = [&](size_t j) -> int {  // results of sub-batch j
        const int s = (int)(j & 1);
        const size_t c0 = sb[j], m = sb[j + 1] - c0;
        P5CHK(hipEventSynchronize(b->evComp[s]));
        const uint64_t* poff = (const uint64_t*)b->hRes[s].p;
        const uint32_t first = *(const uint32_t*)(b->hRes[s].p + up256(8 * (maxN + 1)));
        if (first < m) {
            int32_t st = 0;
            P5CHK(hipMemcpy(&st, b->dMeta[s].p + mStatus + 4 * (size_t)first, 4, hipMemcpyDeviceToHost));
            if (err == PGN_OK) {
                err = st ? st : PGN_ERR_INVALID_ARG;
                errChunk = c0 + first;
            }
            return PGN_OK;
        }
        if (err != PGN_OK) return PGN_OK;
        for (size_t i = 0; i <= m; i++) b->offsets[c0 + i] = outBase + poff[i];
        const uint64_t packed = poff[m];
        P5CHK(hipStreamWaitEvent(b->copy, b->evComp[s], 0));
        if (packed) P5CHK(hipMemcpyAsync(b->hAll.p + outBase, b->dPacked[s].p, packed, hipMemcpyDeviceToHost, b->copy));
        P5CHK(hipEventRecord(b->evD2H[s], b->copy));
        outBase += packed;
        return PGN_OK;
    };
    for (size_t j = 0; j < nsub; j++) {
        const int s = (int)(j & 1);
        const size_t c0 = sb[j], m = sb[j + 1] - c0;
        if (j >= 2) P5CHK(hipEventSynchronize(b->evH2D[s]));  // hIn/hMeta[s] free again
        // samples of the sub-batch's chunks, one job per run of consecutive chunks of a read
        jobs.clear();
        uint64_t at = 0;
        for (size_t i = c0; i < c0 + m;) {
            const uint32_t r = b->readIndex[i];
            size_t e = i;
            uint64_t bytes = 0;
            while (e < c0 + m && b->readIndex[e] == r) bytes += inBytes[e++];
            jobs.push_back({b->hIn[s].p + at, (const uint8_t*)(signal[r] + b->readStart[i]), bytes});
            at += bytes;
            i = e;
        }
        b->pool->run(jobs.data(), jobs.size());
        uint8_t* hm = b->hMeta[s].p;
        uint64_t* hSoff = (uint64_t*)(hm + mSoff);
        uint32_t* hCnt = (uint32_t*)(hm + mCnt);
        uint64_t* hOoff = (uint64_t*)(hm + mOoff);
        uint64_t* hCaps = (uint64_t*)(hm + mCaps);
        uint64_t so = 0, oo = 0;
        for (size_t i = 0; i < m; i++) {
            hSoff[i] = so;
            hCnt[i] = b->samples[c0 + i];
            hOoff[i] = oo;
            hCaps[i] = caps[c0 + i];
            so += b->samples[c0 + i];
            oo += caps[c0 + i];
        }
        if (j >= 2) P5CHK(hipStreamWaitEvent(b->copy, b->evComp[s], 0));  // compute j-2 has read dIn/dMeta[s]
        P5CHK(hipMemcpyAsync(b->dIn[s].p, b->hIn[s].p, at, hipMemcpyHostToDevice, b->copy));
        P5CHK(hipMemcpyAsync(b->dMeta[s].p, hm, mUp, hipMemcpyHostToDevice, b->copy));
        P5CHK(hipEventRecord(b->evH2D[s], b->copy));
        P5CHK(hipStreamWaitEvent(b->stream, b->evH2D[s], 0));
        if (j >= 2) P5CHK(hipStreamWaitEvent(b->stream, b->evD2H[s], 0));  // download j-2 has read dPacked[s]
        uint8_t* dm = b->dMeta[s].p;
        rc = batch_compress(b, m, (const int16_t*)b->dIn[s].p, (const uint64_t*)(dm + mSoff),
                            (const uint32_t*)(dm + mCnt), b->dOut[s].p, (const uint64_t*)(dm + mOoff),
                            (const uint64_t*)(dm + mCaps), (uint64_t*)(dm + mSizes), (int32_t*)(dm + mStatus),
                            b->chunk);
        if (rc) {
            batch_drain(b);
            return rc;
        }
        hipLaunchKernelGGL(pod5_scan_kernel, dim3(1), dim3(1024), 0, b->stream, (const uint64_t*)(dm + mSizes),
                           (const int32_t*)(dm + mStatus), (uint64_t*)(dm + mPoff), (uint32_t*)(dm + mFirst), (uint32_t)m);
        hipLaunchKernelGGL(pod5_pack_kernel, dim3((unsigned)m), dim3(64), 0, b->stream, (const uint8_t*)b->dOut[s].p,
                           (const uint64_t*)(dm + mOoff), (const uint64_t*)(dm + mPoff), b->dPacked[s].p, (uint32_t)m);
        P5CHK(hipGetLastError());
        P5CHK(hipMemcpyAsync(b->hRes[s].p, dm + mPoff, 8 * (m + 1), hipMemcpyDeviceToHost, b->stream));
        P5CHK(hipMemcpyAsync(b->hRes[s].p + up256(8 * (maxN + 1)), dm + mFirst, 4, hipMemcpyDeviceToHost, b->stream));
        P5CHK(hipEventRecord(b->evComp[s], b->stream));
        if (j >= 1 && (rc = finish(j - 1))) {
            batch_drain(b);
            return rc;
        }
    }
    rc = finish(nsub - 1);
    batch_drain(b);
    if (rc) return rc;
    if (err != PGN_OK) {
        *out_chunk_count = errChunk;
        return err;
    }
    *out_chunk_count = n;
    *out_data = b->hAll.p;
    return PGN_OK;
}

// Decompress pipeline over sub-batches of rows, two slots: the blobs -> hIn[s] (copy workers) ->
// dIn[s]; decode into dOut[s]; samples and statuses -> hRes[s]; one sub-batch behind, the copy
// workers move the samples to the caller's buffer while the next sub-batches are in flight.
int pgn_pod5_decompress_rows(pgn_pod5_batch* b, uint32_t row_count, const uint64_t* offsets, const uint8_t* data,
                             const uint32_t* samples, int16_t* out, int32_t* row_status)
{
    if (!b || (row_count && (!offsets || !samples))) return PGN_ERR_INVALID_ARG;
    if (row_count == 0) return PGN_OK;
    const size_t n = row_count;
    if (offsets[n] < offsets[0] || (offsets[n] > offsets[0] && !data)) return PGN_ERR_INVALID_ARG;
    uint64_t total = 0;
    std::vector<uint64_t> inBytes(n);
    for (size_t i = 0; i < n; i++) {
        if (offsets[i + 1] < offsets[i]) return PGN_ERR_INVALID_ARG;
        inBytes[i] = offsets[i + 1] - offsets[i] + 2ull * samples[i] / 4;  // input plus a share of the output
        total += samples[i];
    }
    if (total && !out) return PGN_ERR_INVALID_ARG;
    std::vector<size_t> sb;
    split_subs(inBytes, n, sb);
    const size_t nsub = sb.size() - 1;
    size_t maxIn = 0, maxOut = 0, maxN = 0;
    std::vector<uint64_t> sampleStart(n + 1, 0);
    for (size_t i = 0; i < n; i++) sampleStart[i + 1] = sampleStart[i] + samples[i];
    for (size_t j = 0; j < nsub; j++) {
        const uint64_t a = offsets[sb[j + 1]] - offsets[sb[j]], o = 2 * (sampleStart[sb[j + 1]] - sampleStart[sb[j]]);
        maxIn = a > maxIn ? a : maxIn;
        maxOut = o > maxOut ? o : maxOut;
        maxN = sb[j + 1] - sb[j] > maxN ? sb[j + 1] - sb[j] : maxN;
    }
    // metadata: ioff | isz | soff | cnt (uploaded), status (device, downloaded after the samples)
    const size_t mIoff = 0, mIsz = up256(8 * maxN), mSoff = mIsz + up256(8 * maxN), mCnt = mSoff + up256(8 * maxN),
                 mUp = mCnt + up256(4 * maxN), mStatus = mUp, mAll = mStatus + up256(4 * maxN);
    batch_drain(b);
    int rc;
    for (int s = 0; s < 2 && s < (int)nsub; s++) {
        if ((rc = ensure_pin(b->hIn[s], maxIn)) || (rc = ensure_pin(b->hMeta[s], mUp)) ||
            (rc = ensure_pin(b->hRes[s], up256(maxOut) + up256(4 * maxN))) || (rc = ensure_devbuf(b->dIn[s], maxIn)) ||
            (rc = ensure_devbuf(b->dMeta[s], mAll)) || (rc = ensure_devbuf(b->dOut[s], maxOut)))
            return rc;
    }
    int first = PGN_OK;
    auto finish = [&](size_t j) -> int {  // samples and statuses of sub-batch j to the caller
        const int s = (int)(j & 1);
        const size_t r0 = sb[j], m = sb[j + 1] - r0;
        P5CHK(hipEventSynchronize(b->evD2H[s]));
        const uint64_t ob = 2 * (sampleStart[r0 + m] - sampleStart[r0]);
        const CopyJob job{(uint8_t*)(out + sampleStart[r0]), b->hRes[s].p, ob};
        b->pool->run(&job, 1);
        const int32_t* st = (const int32_t*)(b->hRes[s].p + up256(maxOut));
        for (size_t i = 0; i < m; i++) {
            int32_t sti = st[i];
            if (sti == PGN_ERR_UNSUPPORTED && samples[r0 + i] <= PGN_MAX_CHUNK_SAMPLES) {
                // frames claiming more than the batch's intermediates hold (the bounded call cannot list
                // them without a host wait): the per-chunk call decodes the row as the reference does
                const size_t r = r0 + i;
                const uint8_t* src = data + offsets[r];
                const size_t len = offsets[r + 1] - offsets[r];
                sti = b->codec == PGN_POD5_CODEC_VBZ
                          ? pgn_vbz_decompress_signal(b->ctx, src, len, out + sampleStart[r], samples[r])
                          : pgn_variant_decompress_signal(b->ctx, b->codec, src, len, out + sampleStart[r], samples[r]);
            }
            if (row_status) row_status[r0 + i] = sti;
            if (first == PGN_OK && sti != PGN_OK) first = sti;
        }
        return PGN_OK;
    };
    for (size_t j = 0; j < nsub; j++) {
        const int s = (int)(j & 1);
        const size_t r0 = sb[j], m = sb[j + 1] - r0;
        if (j >= 2) P5CHK(hipEventSynchronize(b->evH2D[s]));
        const uint64_t bytes = offsets[r0 + m] - offsets[r0];
        const CopyJob job{b->hIn[s].p, data + offsets[r0], bytes};
        b->pool->run(&job, 1);
        uint8_t* hm = b->hMeta[s].p;
        uint64_t* hIoff = (uint64_t*)(hm + mIoff);
        uint64_t* hIsz = (uint64_t*)(hm + mIsz);
        uint64_t* hSoff = (uint64_t*)(hm + mSoff);
        uint32_t* hCnt = (uint32_t*)(hm + mCnt);
        uint32_t maxCnt = 0;
        for (size_t i = 0; i < m; i++) {
            hIoff[i] = offsets[r0 + i] - offsets[r0];
            hIsz[i] = offsets[r0 + i + 1] - offsets[r0 + i];
            hSoff[i] = sampleStart[r0 + i] - sampleStart[r0];
            hCnt[i] = samples[r0 + i];
            maxCnt = samples[r0 + i] > maxCnt ? samples[r0 + i] : maxCnt;
        }
        if (j >= 2) P5CHK(hipStreamWaitEvent(b->copy, b->evComp[s], 0));
        if (bytes) P5CHK(hipMemcpyAsync(b->dIn[s].p, b->hIn[s].p, bytes, hipMemcpyHostToDevice, b->copy));
        P5CHK(hipMemcpyAsync(b->dMeta[s].p, hm, mUp, hipMemcpyHostToDevice, b->copy));
        P5CHK(hipEventRecord(b->evH2D[s], b->copy));
        P5CHK(hipStreamWaitEvent(b->stream, b->evH2D[s], 0));
        if (j >= 2) P5CHK(hipStreamWaitEvent(b->stream, b->evD2H[s], 0));  // download j-2 has read dOut[s]
        uint8_t* dm = b->dMeta[s].p;
        rc = batch_decompress(b, m, b->dIn[s].p, (const uint64_t*)(dm + mIoff), (const uint64_t*)(dm + mIsz),
                              (int16_t*)b->dOut[s].p, (const uint64_t*)(dm + mSoff), (const uint32_t*)(dm + mCnt),
                              (int32_t*)(dm + mStatus), maxCnt);
        if (rc) {
            batch_drain(b);
            return rc;
        }
        P5CHK(hipEventRecord(b->evComp[s], b->stream));
        P5CHK(hipStreamWaitEvent(b->copy, b->evComp[s], 0));
        const uint64_t ob = 2 * (sampleStart[r0 + m] - sampleStart[r0]);
        if (ob) P5CHK(hipMemcpyAsync(b->hRes[s].p, b->dOut[s].p, ob, hipMemcpyDeviceToHost, b->copy));
        P5CHK(hipMemcpyAsync(b->hRes[s].p + up256(maxOut), dm + mStatus, 4 * m, hipMemcpyDeviceToHost, b->copy));
        P5CHK(hipEventRecord(b->evD2H[s], b->copy));
        if (j >= 1 && (rc = finish(j - 1))) {
            batch_drain(b);
            return rc;
        }
    }
    rc = finish(nsub - 1);
    batch_drain(b);
    if (rc) return rc;
    return first;
}

static int transcode_impl(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                          int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats,
                          uint32_t flags, pgn_pod5_keep_going_result* kg);

// the host vectors are sized from the file: an allocation failure (or any exception) becomes a
// status instead of crossing the C ABI
int pgn_pod5_transcode_file(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                            int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats)
{
    return pgn_pod5_transcode_file_ex(ctx, in_path, out_path, dst_signal_type, pgnano_variant, rows_per_batch, 0,
                                      stats, nullptr);
}

int pgn_pod5_transcode_file_ex(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                               int pgnano_variant, uint32_t rows_per_batch, uint32_t flags,
                               pgn_pod5_transcode_stats* stats, pgn_pod5_keep_going_result* keep_going)
{
    try {
        return transcode_impl(ctx, in_path, out_path, dst_signal_type, pgnano_variant, rows_per_batch, stats, flags,
                              keep_going);
    } catch (const std::bad_alloc&) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "out of host memory");
        return PGN_ERR_IO;
    } catch (const std::exception& e) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", e.what());
        return PGN_ERR_CORRUPT;
    }
}

}  // extern "C"

// One device pass over a signal column: decode (unless uncompressed), re-encode as dst_signal_type,
// pack on the device, download the packed column.  outOffs gets n + 1 offsets into outData.
// encStatus (keep-going): rows the encoder refuses do not fail the call; their statuses come back
// here (the packed column holds the other rows, a refused row takes no bytes).
static int transcode_rows(pgn_ctx* ctx, int srcType, int dst_signal_type, int pgnano_variant, size_t n,
                          const std::vector<uint32_t>& samples, const std::vector<uint64_t>& offs,
                          const std::vector<uint8_t>& data, uint64_t dataBytes, uint64_t total,
                          std::vector<uint64_t>& outOffs, std::vector<uint8_t>& outData, float& decMs, float& encMs,
                          std::vector<int32_t>* encStatus = nullptr)
{
    if (encStatus) encStatus->assign(n, 0);
    outOffs.assign(n + 1, 0);
    outData.clear();
    decMs = encMs = 0;
    const int srcCodec = srcType == PGN_POD5_SIGNAL_VBZ ? PGN_POD5_CODEC_VBZ : pgnano_variant;
    const int dstCodec = dst_signal_type == PGN_POD5_SIGNAL_VBZ ? PGN_POD5_CODEC_VBZ : pgnano_variant;
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
        uint32_t maxCnt = 0;
        for (size_t i = 0; i < n; i++) maxCnt = samples[i] > maxCnt ? samples[i] : maxCnt;
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
                                     (const uint32_t*)(d + oCnt), (int32_t*)(d + oStatus), maxCnt);
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
                               (const uint64_t*)(d + oCaps), (uint64_t*)(d + oSizes), (int32_t*)(d + oStatus), maxCnt);
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
        if (first < n && encStatus) {
            P5CHK(hipMemcpy(encStatus->data(), d + oStatus, 4 * n, hipMemcpyDeviceToHost));
        } else if (first < n) {
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
    int rc = body();
    if (d) {
        (void)hipStreamSynchronize(stream);
        (void)hipFree(d);
    }
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

static bool transcode_args_ok(pgn_ctx* ctx, int dst_signal_type, int pgnano_variant)
{
    return ctx && dst_signal_type >= PGN_POD5_SIGNAL_UNCOMPRESSED && dst_signal_type <= PGN_POD5_SIGNAL_PGNANO &&
           pgnano_variant >= PGN_VARIANT_C5 && pgnano_variant <= PGN_VARIANT_VBZ0;
}

static int transcode_impl(pgn_ctx* ctx, const char* in_path, const char* out_path, int dst_signal_type,
                          int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats* stats,
                          uint32_t flags, pgn_pod5_keep_going_result* kg)
{
    if (!in_path || !out_path || !transcode_args_ok(ctx, dst_signal_type, pgnano_variant)) return PGN_ERR_INVALID_ARG;
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
    std::vector<uint64_t> offs(rows + 1), outOffs;
    pgn_pod5_signal_read(f, ids.data(), samples.data(), offs.data(), data.data());
    float decMs = 0, encMs = 0;
    const bool keepGoing = (flags & PGN_POD5_KEEP_GOING) != 0;
    std::vector<int32_t> encStatus;
    rc = transcode_rows(ctx, srcType, dst_signal_type, pgnano_variant, (size_t)rows, samples, offs, data, dataBytes,
                        total, outOffs, outData, decMs, encMs, keepGoing ? &encStatus : nullptr);
    if (rc == PGN_OK) {
        if (keepGoing) {
            pgn_pod5_keep_going_result r{};
            rc = pgn_pod5_write_file_keep_going(out_path, f, dst_signal_type, rows, ids.data(), samples.data(),
                                                outOffs.data(), outData.data(), encStatus.data(), rows_per_batch,
                                                nullptr, &r);
            if (kg) *kg = r;
        } else {
            rc = pgn_pod5_write_file(out_path, f, dst_signal_type, rows, ids.data(), samples.data(), outOffs.data(),
                                     outData.data(), rows_per_batch, nullptr, nullptr);
        }
        if (rc) snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", pgn_pod5_file_error());
    }
    if (rc == PGN_OK && stats) {
        stats->rows = rows;
        stats->samples = total;
        stats->in_bytes = dataBytes;
        stats->out_bytes = outOffs[rows];
        stats->decode_ms = decMs;
        stats->encode_ms = encMs;
    }
    pgn_pod5_file_close(f);
    return rc;
}

struct pgn_pod5_part {
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> data;
};

static int transcode_part_impl(pgn_ctx* ctx, const pgn_pod5_file* f, const uint32_t* batch_ids, uint32_t nIds,
                               int dst_signal_type, int pgnano_variant, pgn_pod5_part** out,
                               pgn_pod5_transcode_stats* stats)
{
    if (!f || !out || (nIds && !batch_ids) || !transcode_args_ok(ctx, dst_signal_type, pgnano_variant))
        return PGN_ERR_INVALID_ARG;
    *out = nullptr;
    uint64_t rows = 0, dataBytes = 0, total = 0, allRows = 0;
    uint32_t nb = 0;
    int srcType = 0;
    pgn_pod5_signal_info(f, &allRows, &nb, &srcType, nullptr, nullptr);
    int rc = pgn_pod5_signal_read_batches(f, batch_ids, nIds, &rows, &dataBytes, &total, nullptr, nullptr, nullptr,
                                          nullptr);
    if (rc) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "batch id out of range (%u record batches)", nb);
        return rc;
    }
    std::vector<uint8_t> data(dataBytes);
    std::vector<uint32_t> samples(rows);
    std::vector<uint64_t> offs(rows + 1);
    pgn_pod5_signal_read_batches(f, batch_ids, nIds, nullptr, nullptr, nullptr, nullptr, samples.data(), offs.data(),
                                 data.data());
    std::unique_ptr<pgn_pod5_part> part(new pgn_pod5_part);
    float decMs = 0, encMs = 0;
    rc = transcode_rows(ctx, srcType, dst_signal_type, pgnano_variant, (size_t)rows, samples, offs, data, dataBytes,
                        total, part->offsets, part->data, decMs, encMs);
    if (rc) return rc;
    if (stats) {
        stats->rows = rows;
        stats->samples = total;
        stats->in_bytes = dataBytes;
        stats->out_bytes = part->offsets[rows];
        stats->decode_ms = decMs;
        stats->encode_ms = encMs;
    }
    *out = part.release();
    return PGN_OK;
}

extern "C" {

int pgn_pod5_transcode_part(pgn_ctx* ctx, const pgn_pod5_file* f, const uint32_t* batch_ids, uint32_t n,
                            int dst_signal_type, int pgnano_variant, pgn_pod5_part** out,
                            pgn_pod5_transcode_stats* stats)
{
    try {
        return transcode_part_impl(ctx, f, batch_ids, n, dst_signal_type, pgnano_variant, out, stats);
    } catch (const std::bad_alloc&) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "out of host memory");
        return PGN_ERR_IO;
    } catch (const std::exception& e) {
        snprintf(g_pod5_err, sizeof(g_pod5_err), "%s", e.what());
        return PGN_ERR_CORRUPT;
    }
}

int pgn_pod5_part_get(const pgn_pod5_part* part, uint64_t* rows, const uint64_t** offsets, const uint8_t** data)
{
    if (!part) return PGN_ERR_INVALID_ARG;
    if (rows) *rows = part->offsets.size() - 1;
    if (offsets) *offsets = part->offsets.data();
    if (data) *data = part->data.data();
    return PGN_OK;
}

int pgn_pod5_part_free(pgn_pod5_part* part)
{
    delete part;
    return PGN_OK;
}

}  // extern "C"


