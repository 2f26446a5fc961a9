/*
 * pgnano_hip.h -- C ABI of the MI355X (gfx950) pgnano "C5" signal codec.
 *
 * Drop-in boundary for the reference's per-chunk plugin surface (tomas-gr/RawNanoporeSignalCompression):
 *   pgnano::compress_signal   pod5/c++/pod5_format/pgnano/pgnano.h:19-23, pgnano.cpp:59-96
 *   pgnano::decompress_signal pod5/c++/pod5_format/pgnano/pgnano.h:13-17, pgnano.cpp:98-126
 * and of the pod5 C-API entry points built on it (pod5/c++/pod5_format/c_api.h:676-712,
 * c_api.cpp:1177-1273).  The compressed bytes are identical to the reference's default
 * COMPRESSOR_C5 variant (pgnano/svb16/C5.hpp:282-683) with libzstd 1.4.8/1.4.9 level 1.
 *
 * Plain pointers and sizes only.  Functions taking `d_` pointers expect device (HBM) memory and are
 * asynchronous on the given HIP stream (`stream` is a hipStream_t, NULL = the context's stream);
 * the others take host memory and are synchronous.  Every function returns a pgn_status.
 */
#ifndef PGNANO_HIP_H
#define PGNANO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum pgn_status {
    PGN_OK = 0,
    PGN_ERR_DST_TOO_SMALL = 1,    /* "Not enough space in destination buffer"       C5.hpp:420-427 */
    PGN_ERR_NOT_ZSTD = 2,         /* "Input data not compressed by zstd"            C5.hpp:495-502 */
    PGN_ERR_ZSTD_DECOMPRESS = 3,  /* "Input data failed to decompress using zstd"   C5.hpp:593-600 */
    PGN_ERR_REMAINING = 4,        /* "Remaining data at end of signal buffer"       C5.hpp:675-677 */
    PGN_ERR_ZSTD_COMPRESS = 5,    /* "Failed to compress ..."                        C5.hpp:340-342 */
    PGN_ERR_CORRUPT = 6,          /* input on which the reference reads out of bounds (UB there) */
    PGN_ERR_ALLOC = 8,            /* decode: the frames' content sizes sum to more than 2^40 bytes, taken as the
                                     reference's allocation of that intermediate failing (C5.hpp:575-583); also
                                     a chunk whose frames could really expand to more than 1 GiB (the claims pass's
                                     intermediate limit, see the decode notes below) */
    PGN_ERR_UNSUPPORTED = 9,      /* chunk above PGN_MAX_CHUNK_SAMPLES */
    PGN_ERR_INVALID_ARG = 10,
    PGN_ERR_HIP = 11,             /* HIP runtime failure (message in pgn_last_error) */
    PGN_ERR_NO_DEVICE = 12,
    PGN_ERR_IO = 13               /* file open/read/write failure (pgnano_pod5file.h) */
} pgn_status;

/* Largest chunk the GPU path encodes and decodes (16 Mi samples; the reference takes any size: its
 * ZSTD_compress and svb16 calls are unbounded, signal_compression.cpp:57-66, C5.hpp:337-413).  Every
 * stream is one zstd frame in 128 KiB blocks as libzstd 1.4.x writes it at level 1: single-segment
 * up to 512 KiB, a window-descriptor frame (windowLog 19, matches within the window) above.  The
 * reference writer's default chunk is 102,400 samples (pod5/c++/pod5_format/file_writer.h:22); the
 * chunk size is a writer option (c_api.h:526-539).
 * Chunks up to 262,144 samples run in the batched passes; larger ones in a second pass of the same
 * call whose per-chunk buffers are spaced for the largest of them (see the batch calls below).
 * Decode: a chunk's decoded frames share an intermediate buffer of 2.25 bytes per sample + 1,024 of
 * the call's largest chunk (262,144 samples when the call gives no bound): every blob whose frames
 * decode to what its merge consumes fits it.  Frames whose content sizes claim more are decoded as the
 * reference decodes them -- each into exactly its claim, in an intermediate of the claims' sum -- by a
 * second pass of the same call (a claim the frame's blocks cannot produce is "failed to decompress",
 * as ZSTD_decompress reports it, without decoding); so a chunk's status does not depend on the other
 * chunks of its call. */
#define PGN_MAX_CHUNK_SAMPLES 16777216u

/* Per-chunk statistics, the reference's global byte counters (src/c++/copy.cpp:64-85, updated at
 * C5.hpp:318-324,467-471): raw stream sizes then frame sizes, order keys, S, M, Llow, Lhigh. */
#define PGN_STATS_PER_CHUNK 10

typedef struct pgn_ctx pgn_ctx;

/* Message of a status code (the reference's arrow::Status text where one exists). */
const char *pgn_status_string(int status);
/* Detail of the last PGN_ERR_HIP on this thread. */
const char *pgn_last_error(void);

/* Context bound to one HIP device (one process per GPU): scratch memory and a stream. */
int pgn_ctx_create(int device, pgn_ctx **out);
int pgn_ctx_destroy(pgn_ctx *ctx);
/* The context's HIP stream (hipStream_t). */
void *pgn_ctx_stream(pgn_ctx *ctx);

/* pgnano::Compressor::compressed_signal_max_size (pgnano/compressor.h:39-45):
 * max(2n + 26, 1024) -- the destination size pgnano::compress_signal allocates. */
size_t pgn_compressed_signal_max_size(size_t sample_count);

/* pgnano::compress_signal (pgnano.cpp:59-96) -> compress_signal_N01 (C5.hpp:282-474), host memory.
 * dst_capacity plays the role of the destination span; *out_size gets the blob size (or, on
 * PGN_ERR_DST_TOO_SMALL, the required size the reference prints at C5.hpp:423-424). */
int pgn_compress_signal(pgn_ctx *ctx, const int16_t *samples, size_t sample_count, uint8_t *dst,
                        size_t dst_capacity, size_t *out_size);

/* pgnano::decompress_signal (pgnano.cpp:98-126) -> decompress_signal_N01 (C5.hpp:477-683), host
 * memory; sample_count is the destination span size (the POD5 `samples` column). */
int pgn_decompress_signal(pgn_ctx *ctx, const uint8_t *compressed, size_t compressed_size, int16_t *dst,
                          size_t sample_count);

/* pod5_pinanoraw_compress_signal (c_api.h:696-700, c_api.cpp:1217-1253) on a default context of
 * device 0: *compressed_signal_size is the buffer size on input, the blob size on output. */
int pgn_pinanoraw_compress_signal(const int16_t *signal, size_t signal_size, char *compressed_signal_out,
                                  size_t *compressed_signal_size);

/* pod5_vbz_compress_signal / pod5_vbz_decompress_signal (c_api.h:685-711, c_api.cpp:1183-1214,
 * 1255-1273) with the same argument shapes, on the default context of device 0: the VBZ codec of
 * the reference's --VBZ path.  Compress: *compressed_signal_size is the buffer size on input and
 * the blob size on output (a blob larger than the buffer is PGN_ERR_DST_TOO_SMALL, the reference's
 * "Compressed signal size (..) is greater than provided buffer size").  Decompress: sample_count
 * samples into signal_out. */
int pgn_pod5_vbz_compress_signal(const int16_t *signal, size_t signal_size, char *compressed_signal_out,
                                 size_t *compressed_signal_size);
int pgn_pod5_vbz_decompress_signal(const char *compressed_signal, size_t compressed_signal_size,
                                   size_t sample_count, short *signal_out);

/* Batched, device-resident encode of `nchunks` independent chunks (each <= PGN_MAX_CHUNK_SAMPLES):
 * chunk i = d_samples[d_sample_offsets[i] .. + d_sample_counts[i]) -> d_out[d_out_offsets[i] ..),
 * capacity d_out_caps[i]; d_out_sizes[i] and d_status[i] receive the result.  d_stats (optional)
 * receives PGN_STATS_PER_CHUNK uint64 per chunk.
 * The batch calls are asynchronous on `stream` except for one host wait: the chunks above 262,144
 * samples (and, when decoding, the chunks whose frames claim more than the batched pass's
 * intermediates) are listed by a small kernel that runs after the work queued before the call (while
 * the batched pass runs) and the host reads their count before queueing their pass.  The wait ends
 * when the earlier work and that kernel have finished, not the call's own kernels.  The _bounded
 * variants below skip it. */
int pgn_compress_batch_device(pgn_ctx *ctx, size_t nchunks, const int16_t *d_samples,
                              const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts, uint8_t *d_out,
                              const uint64_t *d_out_offsets, const uint64_t *d_out_caps, uint64_t *d_out_sizes,
                              int32_t *d_status, uint64_t *d_stats, void *stream);

/* Batched, device-resident decode: blob i = d_in[d_in_offsets[i] .. + d_in_sizes[i]) ->
 * d_samples[d_sample_offsets[i] .. + d_sample_counts[i]). */
int pgn_decompress_batch_device(pgn_ctx *ctx, size_t nchunks, const uint8_t *d_in, const uint64_t *d_in_offsets,
                                const uint64_t *d_in_sizes, int16_t *d_samples, const uint64_t *d_sample_offsets,
                                const uint32_t *d_sample_counts, int32_t *d_status, void *stream);

/* The batch calls with the caller's bound on the chunk sizes (max_chunk_samples >= every
 * d_sample_counts[i], e.g. the writer's chunk size, file_writer.h:22): with a bound at or below
 * 262,144 samples no scan runs and the call never waits on the host; the decode intermediates are
 * spaced for the bound.  A chunk above the bound may get PGN_ERR_UNSUPPORTED.  Decode: a chunk whose
 * frames claim more than 2.25 x the bound + 1,024 bytes and could really produce it gets
 * PGN_ERR_UNSUPPORTED here (listing it needs the host wait; the unbounded call decodes it as the
 * reference does). */
int pgn_compress_batch_device_bounded(pgn_ctx *ctx, uint32_t max_chunk_samples, size_t nchunks,
                                      const int16_t *d_samples, const uint64_t *d_sample_offsets,
                                      const uint32_t *d_sample_counts, uint8_t *d_out, const uint64_t *d_out_offsets,
                                      const uint64_t *d_out_caps, uint64_t *d_out_sizes, int32_t *d_status,
                                      uint64_t *d_stats, void *stream);
int pgn_decompress_batch_device_bounded(pgn_ctx *ctx, uint32_t max_chunk_samples, size_t nchunks, const uint8_t *d_in,
                                        const uint64_t *d_in_offsets, const uint64_t *d_in_sizes, int16_t *d_samples,
                                        const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts,
                                        int32_t *d_status, void *stream);

/* ---- VBZ: the pod5 baseline codec (svb16 + zstd level 1), same context, same conventions ------
 * pod5::compressed_signal_max_size (signal_compression.cpp:14-19):
 * ZSTD_compressBound(svb16_max_encoded_length(n)) = ZSTD_compressBound(ceil(n/8) + 2n). */
size_t pgn_vbz_compressed_signal_max_size(size_t sample_count);

/* pod5::compress_signal(samples, pool, destination) (signal_compression.cpp:21-50): the compressed
 * size in *out_size; a frame larger than dst_capacity is PGN_ERR_ZSTD_COMPRESS ("Failed to compress
 * data"). */
int pgn_vbz_compress_signal(pgn_ctx *ctx, const int16_t *samples, size_t sample_count, uint8_t *dst,
                            size_t dst_capacity, size_t *out_size);

/* pod5::decompress_signal(compressed, pool, destination) (signal_compression.cpp:96-141). */
int pgn_vbz_decompress_signal(pgn_ctx *ctx, const uint8_t *compressed, size_t compressed_size, int16_t *dst,
                              size_t sample_count);

/* Batched device-resident VBZ encode / decode; arguments as pgn_compress_batch_device /
 * pgn_decompress_batch_device (d_stats: svb16 bytes at [0], frame bytes at [5], others 0). */
int pgn_vbz_compress_batch_device(pgn_ctx *ctx, size_t nchunks, const int16_t *d_samples,
                                  const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts, uint8_t *d_out,
                                  const uint64_t *d_out_offsets, const uint64_t *d_out_caps, uint64_t *d_out_sizes,
                                  int32_t *d_status, uint64_t *d_stats, void *stream);
int pgn_vbz_decompress_batch_device(pgn_ctx *ctx, size_t nchunks, const uint8_t *d_in, const uint64_t *d_in_offsets,
                                    const uint64_t *d_in_sizes, int16_t *d_samples, const uint64_t *d_sample_offsets,
                                    const uint32_t *d_sample_counts, int32_t *d_status, void *stream);

/* ---- The other compile-time pgnano variants as a runtime choice ------------------------------
 * The reference builds one binary per `#define COMPRESSOR_*` (pgnano.cpp:1, 70-92, 105-125;
 * utils/compile_all.sh); blobs carry no variant tag, so reader and writer must agree on it.  Same
 * conventions as the C5 entry points (destination capacity max(2n+26, 1024) from
 * pgn_compressed_signal_max_size; C5 through these calls equals the C5 functions above).
 *   C4   compress_signal_N02    (pgnano/svb16/C4.hpp:274-679)    5 frames, C5 layout on raw values
 *   C1   compress_signal_KD     (C1.hpp:202-382)                 2 frames: svb16 keys, svb16 data
 *   C2   compress_signal_lh     (C2.hpp:195-463)                 3 frames: keys, low bytes, high bytes
 *   C3   compress_signal_ll_lh  (C3.hpp:212-503)                 4 frames: keys, small low, big low, big high
 *   VBZ0 compress_signal_VBZ1   (VBZ_0.hpp:316-423)              1 frame: 2-bit keys + nibble stream
 * VBZ0 compresses straight into the destination ("Failed to compress data" = PGN_ERR_ZSTD_COMPRESS
 * when the frame does not fit); C1/C2/C3 copy into it unchecked in the reference, here a
 * too-small destination is PGN_ERR_DST_TOO_SMALL with the required size, as for C5/C4. */
typedef enum pgn_variant {
    PGN_VARIANT_C5 = 0,
    PGN_VARIANT_C4 = 1,
    PGN_VARIANT_C1 = 2,
    PGN_VARIANT_C2 = 3,
    PGN_VARIANT_C3 = 4,
    PGN_VARIANT_VBZ0 = 5
} pgn_variant;

int pgn_variant_compress_signal(pgn_ctx *ctx, int variant, const int16_t *samples, size_t sample_count, uint8_t *dst,
                                size_t dst_capacity, size_t *out_size);
int pgn_variant_decompress_signal(pgn_ctx *ctx, int variant, const uint8_t *compressed, size_t compressed_size,
                                  int16_t *dst, size_t sample_count);
/* d_stats: raw stream sizes at [0..frames), frame sizes at [5..5+frames), in frame order */
int pgn_variant_compress_batch_device(pgn_ctx *ctx, int variant, size_t nchunks, const int16_t *d_samples,
                                      const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts,
                                      uint8_t *d_out, const uint64_t *d_out_offsets, const uint64_t *d_out_caps,
                                      uint64_t *d_out_sizes, int32_t *d_status, uint64_t *d_stats, void *stream);
int pgn_variant_decompress_batch_device(pgn_ctx *ctx, int variant, size_t nchunks, const uint8_t *d_in,
                                        const uint64_t *d_in_offsets, const uint64_t *d_in_sizes, int16_t *d_samples,
                                        const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts,
                                        int32_t *d_status, void *stream);

/* Device generator of the synthetic nanopore-like reads used by bench.py (integer-only, identical
 * to the checker's pgno_synth_read): global read first_read + r * read_stride ->
 * d_samples[d_sample_offsets[r] .. + d_sample_counts[r]). */
int pgn_synth_reads_device(pgn_ctx *ctx, size_t nreads, uint64_t seed, uint64_t first_read, uint64_t read_stride,
                           int16_t *d_samples,
                           const uint64_t *d_sample_offsets, const uint32_t *d_sample_counts,
                           uint32_t p_switch_q16, int32_t level_mean, int32_t level_sd, int32_t noise_sd, void *stream);

/* Diagnostics: accumulated shader-clock cycles per kernel phase (out[0..15] encode, out[16..31]
 * decode; all zero unless the context was created with PGN_PHASE_PROFILE=1 in the environment). */
int pgn_debug_phase_cycles(pgn_ctx *ctx, uint64_t *out, int n);
/* Diagnostics: per-stream decode records of the first n chunks of the last decode pass
 * (5 per chunk, 24 bytes each: u64 frame offset, u32 frame bytes, u32 content size,
 * u32 intermediate offset, i32 decoded bytes or a negative error). */
int pgn_debug_decode_units(pgn_ctx *ctx, void *out, size_t nchunks);

/* Kernels of the C5 batch path on ctx, direction 0 = encode, 1 = decode: the fused per-chunk kernel
 * or the staged three-kernel pipeline (PGN_ENC_PIPELINE / PGN_DEC_PIPELINE = fused | staged). */
const char *pgn_ctx_kernels(pgn_ctx *ctx, int direction);

/* Kernel time (ms, HIP events on the launch stream) of the last batch encode / decode call on ctx. */
float pgn_ctx_last_encode_ms(pgn_ctx *ctx);
float pgn_ctx_last_decode_ms(pgn_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* PGNANO_HIP_H */
