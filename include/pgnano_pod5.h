/*
 * pgnano_pod5.h -- batched POD5 signal-table integration of the MI355X pgnano / VBZ codecs (C ABI).
 *
 * The reference's writer hands a whole batch of reads to the library at once
 *   pod5_add_reads_data(file, read_count, ..., int16_t const ** signal, uint32_t const * signal_size)
 *     (pod5/c++/pod5_format/c_api.cpp:1104-1129)
 * and then chunks every read at the writer's max_signal_chunk_size (default 102,400,
 * file_writer.h:22; chunking loop file_writer.cpp:119-143), compressing one chunk per call
 * (signal_table_writer.cpp:105-112) into the signal table's (offsets, data) column.  The reader
 * decodes the rows of a signal record batch one by one (signal_table_reader.cpp:294-318).
 *
 * Here the same work is done per batch: every chunk of every read of a pod5_add_reads_data call is
 * compressed by one batched GPU launch, and the result is returned in the signal column layout
 * the writer appends (blob i = data[offsets[i] .. offsets[i + 1]), samples[i] samples, read
 * read_index[i]); a reader batch of rows is decoded by one batched launch.  Host memory in and out
 * (the transfers to and from HBM happen inside, through pinned staging buffers that the batch
 * object keeps).  The bytes are those of the per-chunk entry points in pgnano_hip.h.
 */
#ifndef PGNANO_POD5_H
#define PGNANO_POD5_H

#include <stddef.h>
#include <stdint.h>

#include "pgnano_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* file_writer.h:22 DEFAULT_SIGNAL_CHUNK_SIZE */
#define PGN_POD5_DEFAULT_CHUNK_SIZE 102400u

/* Codec of a batch: a pgnano variant (pgn_variant, PGN_VARIANT_C5 = the reference default) or the
 * pod5 VBZ codec (--VBZ). */
#define PGN_POD5_CODEC_VBZ 100

typedef struct pgn_pod5_batch pgn_pod5_batch;

/* Detail of the last failure of a pgn_pod5_* call on this thread (HIP error, failing row). */
const char *pgn_pod5_last_error(void);

/* A batch object on `ctx` (which it does not own) for one codec and chunk size (0 = the writer's
 * default, at most PGN_MAX_CHUNK_SAMPLES).  It keeps its staging buffers between calls. */
int pgn_pod5_batch_create(pgn_ctx *ctx, int codec, uint32_t chunk_size, pgn_pod5_batch **out);
int pgn_pod5_batch_destroy(pgn_pod5_batch *batch);

/* pod5_add_reads_data's signal half: read r (signal[r], signal_size[r] samples) becomes
 * ceil(signal_size[r] / chunk_size) chunks (none for an empty read), in read order.  On PGN_OK:
 *   *out_chunk_count      chunks of the batch;
 *   *out_offsets          chunk_count + 1 byte offsets into *out_data (the column's offsets);
 *   *out_data             the compressed chunks back to back (the column's data);
 *   *out_samples          samples per chunk (the signal table's `samples` column);
 *   *out_read_index       the read each chunk belongs to.
 * The arrays are owned by the batch and valid until its next call.  A chunk the codec refuses
 * (pgnano: "Not enough space in destination buffer", VBZ: "Failed to compress data") fails the
 * call with that status; *out_chunk_count is then the index of the first failing chunk. */
int pgn_pod5_compress_reads(pgn_pod5_batch *batch, uint32_t read_count, const int16_t *const *signal,
                            const uint32_t *signal_size, size_t *out_chunk_count, const uint64_t **out_offsets,
                            const uint8_t **out_data, const uint32_t **out_samples, const uint32_t **out_read_index);

/* A record batch of signal rows (signal_table_reader.cpp:294-318): row i = data[offsets[i] ..
 * offsets[i + 1]) decodes to samples[i] samples, written back to back into out (room for the sum
 * of samples[]).  row_status (optional, row_count entries) receives each row's pgn_status; the
 * call returns the first non-zero row status, else PGN_OK.  A row whose frames claim more content
 * than the batch's intermediates hold is decoded again by the per-chunk call (its frames into exactly
 * their claims, as the reference decodes them), so its status is the reference's. */
int pgn_pod5_decompress_rows(pgn_pod5_batch *batch, uint32_t row_count, const uint64_t *offsets, const uint8_t *data,
                             const uint32_t *samples, int16_t *out, int32_t *row_status);

#ifdef __cplusplus
}
#endif

#endif /* PGNANO_POD5_H */
