// pgn_internal.h -- in-library entry points shared by pgn_kernels.hip and pgn_pod5.hip (not part of
// the C ABI).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/pgnano_hip.h"

// The batched device calls of pgnano_hip.h for a pgnano variant (pgn_variant) or the VBZ codec
// (PGN_POD5_CODEC_VBZ), with the caller's bound on d_sample_counts (max_samples, 0 = unknown): a
// bound at or below the batched passes' chunk size skips the large-chunk scan and its host wait.
__attribute__((visibility("hidden"))) int pgn_compress_batch_bounded(
    pgn_ctx* ctx, int codec, uint32_t max_samples, size_t nchunks, const int16_t* d_samples,
    const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts, uint8_t* d_out, const uint64_t* d_out_offsets,
    const uint64_t* d_out_caps, uint64_t* d_out_sizes, int32_t* d_status, uint64_t* d_stats, void* stream);
__attribute__((visibility("hidden"))) int pgn_decompress_batch_bounded(
    pgn_ctx* ctx, int codec, uint32_t max_samples, size_t nchunks, const uint8_t* d_in, const uint64_t* d_in_offsets,
    const uint64_t* d_in_sizes, int16_t* d_samples, const uint64_t* d_sample_offsets, const uint32_t* d_sample_counts,
    int32_t* d_status, void* stream);
