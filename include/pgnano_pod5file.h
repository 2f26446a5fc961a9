/*
 * pgnano_pod5file.h -- POD5 container I/O for the signal table, without Arrow (C ABI).
 *
 * A POD5 file is a "combined file" (pod5/docs/SPECIFICATION.md "Combined file Layout"):
 *   <signature "\213POD\r\n\032\n"> <section marker, 16 bytes>
 *   <embedded Arrow IPC file (padded to 8 bytes)> <section marker> ...
 *   <"FOOTER\0\0"> <footer flatbuffer (padded to 8)> <int64 footer length> <section marker> <signature>
 * The footer (pod5/c++/pod5_format/flatbuffers/footer.fbs) lists the embedded files: the signal
 * table, the run-info table and the reads table (written in that order by file_writer.cpp:300-350,
 * footer by internal/combined_file_utils.h:85-151, read back by combined_file_utils.h:188-279).
 * The signal table (signal_table_schema.cpp:15-42) has three columns: read_id (minknow.uuid,
 * fixed_size_binary(16)), signal (minknow.vbz or pgnano.signal over large_binary, or
 * large_list<int16> uncompressed) and samples (uint32), in record batches of 100 rows
 * (file_writer.h:23 DEFAULT_SIGNAL_TABLE_BATCH_SIZE).
 *
 * This header replaces the Arrow-based pieces of that path with a native reader and writer: the
 * footer and the Arrow IPC file format (flatbuffer schema, record batch and footer messages) are
 * parsed and written directly, so the signal column can be handed to the GPU codec without Arrow.
 * The other embedded tables are not interpreted: a writer given a source file copies them byte for
 * byte (what the reference's `copy` does to them when only the signal codec changes).
 *
 * pgn_pod5_transcode_file (GPU) is `copy in.pod5 out.pod5 --pgnano | --VBZ` for the signal table:
 * the rows are decoded and re-encoded by batched launches (pgnano_pod5.h's codecs) and written with
 * the source's row order, read ids, reads and run-info tables.
 */
#ifndef PGNANO_POD5FILE_H
#define PGNANO_POD5FILE_H

#include <stddef.h>
#include <stdint.h>

#include "pgnano_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* footer.fbs ContentType */
#define PGN_POD5_CONTENT_READS 0
#define PGN_POD5_CONTENT_SIGNAL 1
#define PGN_POD5_CONTENT_READ_ID_INDEX 2
#define PGN_POD5_CONTENT_OTHER_INDEX 3
#define PGN_POD5_CONTENT_RUN_INFO 4

/* signal_table_utils.h:5 SignalType */
#define PGN_POD5_SIGNAL_UNCOMPRESSED 0
#define PGN_POD5_SIGNAL_VBZ 1
#define PGN_POD5_SIGNAL_PGNANO 2

/* file_writer.h:23 */
#define PGN_POD5_DEFAULT_SIGNAL_BATCH_ROWS 100u

typedef struct pgn_pod5_file pgn_pod5_file;

/* Text of the last failure of a pgn_pod5_file_* / pgn_pod5_write_* call on this thread. */
const char *pgn_pod5_file_error(void);

/* Opens a combined POD5 file: checks both signatures, parses the footer and the signal table's
 * schema and record-batch index (combined_file_utils.h:188-279, signal_table_schema.cpp:45-80).
 * PGN_ERR_CORRUPT for a malformed file, PGN_ERR_UNSUPPORTED for body-compressed or null-bearing
 * signal batches. */
int pgn_pod5_file_open(const char *path, pgn_pod5_file **out);
int pgn_pod5_file_close(pgn_pod5_file *f);

/* Footer strings (valid while f is open). */
const char *pgn_pod5_file_identifier(const pgn_pod5_file *f);
const char *pgn_pod5_file_software(const pgn_pod5_file *f);
const char *pgn_pod5_file_pod5_version(const pgn_pod5_file *f);

/* The footer's embedded files, in footer order. */
int pgn_pod5_file_embedded_count(const pgn_pod5_file *f);
int pgn_pod5_file_embedded(const pgn_pod5_file *f, int index, int64_t *offset, int64_t *length, int *content_type);

/* Signal table shape: rows, record batches, the signal type (PGN_POD5_SIGNAL_*), the bytes of the
 * signal column's data (compressed bytes, or 2 x samples when uncompressed) and the sum of the
 * samples column. */
int pgn_pod5_signal_info(const pgn_pod5_file *f, uint64_t *rows, uint32_t *batches, int *signal_type,
                         uint64_t *data_bytes, uint64_t *total_samples);

/* Copies the signal table out, all batches in order (any pointer may be NULL to skip a column):
 *   read_ids  16 x rows bytes;  samples  rows entries;
 *   offsets   rows + 1 byte offsets into data (offsets[0] = 0);  data  data_bytes bytes
 *   (little-endian int16 samples when the table is uncompressed). */
int pgn_pod5_signal_read(const pgn_pod5_file *f, uint8_t *read_ids, uint32_t *samples, uint64_t *offsets,
                         uint8_t *data);

/* The rows of signal record batch `batch`: rows first_row .. first_row + rows - 1 of the table. */
int pgn_pod5_signal_batch_rows(const pgn_pod5_file *f, uint32_t batch, uint64_t *first_row, uint64_t *rows);

/* The rows of the record batches batch_ids[0 .. n), in that order, copied out as
 * pgn_pod5_signal_read does (offsets relative to this selection; any array may be NULL).  With the
 * arrays NULL it reports the selection's rows, data bytes and samples, to size them. */
int pgn_pod5_signal_read_batches(const pgn_pod5_file *f, const uint32_t *batch_ids, uint32_t n, uint64_t *rows,
                                 uint64_t *data_bytes, uint64_t *total_samples, uint8_t *read_ids, uint32_t *samples,
                                 uint64_t *offsets, uint8_t *data);

/* Writes a combined POD5 file whose signal table holds the given rows (row i: read_ids[16 i ..],
 * samples[i], signal bytes data[offsets[i] .. offsets[i + 1])) as `signal_type`, in record batches
 * of rows_per_batch rows (0 = 100).
 * With `source` (may be NULL): the footer's file identifier, software and pod5 version and the
 * signal table's schema metadata are the source's, and every embedded table of the source other
 * than its signal table is copied byte for byte after the signal table, in footer order.
 * Without: a signal-table-only file with a fresh file identifier, `software` (NULL =
 * "rawnanoporesignalcompression_amd") and pod5 version "0.3.10".
 * section_marker: 16 bytes, or NULL for a random one. */
int pgn_pod5_write_file(const char *path, const pgn_pod5_file *source, int signal_type, uint64_t rows,
                        const uint8_t *read_ids, const uint32_t *samples, const uint64_t *offsets, const uint8_t *data,
                        uint32_t rows_per_batch, const char *software, const uint8_t *section_marker);

/* The layout pgn_pod5_write_file gives the same arguments, with the signal bytes left zero so that
 * other processes can write them in place: row_positions[i] (rows entries, may be NULL) receives the
 * file offset of row i's signal bytes.  write = 0 only computes the positions (path may be NULL);
 * every process that calls it with the same arguments gets the same positions.  Used by the
 * multi-GPU copy: rank 0 writes the file, every rank writes its own rows at their positions, so
 * only sizes cross the collective.  section_marker must be given when the positions are used (the
 * marker does not move them, but a random one would make the ranks' files differ). */
int pgn_pod5_write_file_reserved(const char *path, const pgn_pod5_file *source, int signal_type, uint64_t rows,
                                 const uint8_t *read_ids, const uint32_t *samples, const uint64_t *offsets,
                                 uint32_t rows_per_batch, const char *software, const uint8_t *section_marker,
                                 int write, uint64_t *row_positions);

/* Keep-going copy (the reference's `copy` after a failing read, src/c++/copy.cpp:174-176): the rows
 * whose row_status is not 0 could not be written.  Read batch by read batch of the source's reads
 * table, read by read: a read's signal rows are written up to its first failing row; that read and
 * the rest of its read batch are not written (pod5_add_reads_data stops at the failing read,
 * pod5/c++/pod5_format/c_api.cpp:1118-1127); the rows written before the failing one stay in the
 * signal table, listed by no read.  The reads table is rewritten with the kept reads and their
 * signal rows renumbered (its dictionaries and schema copied byte for byte); with no failing row
 * the file is the one pgn_pod5_write_file writes.  Rows no read lists are written when they
 * transcoded.  Without a reads table (or source) every failing row is dropped on its own. */
typedef struct pgn_pod5_keep_going_result {
    uint64_t failed_batches;    /* read batches cut short */
    uint64_t dropped_reads;     /* reads not written */
    uint64_t dropped_rows;      /* signal rows not written */
    uint64_t orphan_rows;       /* rows written before a failing row of their read (listed by no read) */
    uint64_t first_failed_row;  /* input signal row of the first failure in read order; UINT64_MAX if none */
    int32_t first_status;
    int32_t pad;
} pgn_pod5_keep_going_result;
int pgn_pod5_write_file_keep_going(const char *path, const pgn_pod5_file *source, int signal_type, uint64_t rows,
                                   const uint8_t *read_ids, const uint32_t *samples, const uint64_t *offsets,
                                   const uint8_t *data, const int32_t *row_status, uint32_t rows_per_batch,
                                   const uint8_t *section_marker, pgn_pod5_keep_going_result *res);

/* The row count of every signal record batch (counts: one entry per batch). */
int pgn_pod5_signal_batch_row_counts(const pgn_pod5_file *f, uint64_t *counts);

typedef struct pgn_pod5_transcode_stats {
    uint64_t rows;
    uint64_t samples;
    uint64_t in_bytes;   /* signal column data of the input */
    uint64_t out_bytes;  /* signal column data written */
    float decode_ms;     /* device time of the batched decode (0 when the input is uncompressed) */
    float encode_ms;     /* device time of the batched encode (0 when the output is uncompressed) */
} pgn_pod5_transcode_stats;

/* `copy in.pod5 out.pod5 --pgnano | --VBZ` on the GPU for the signal table: every row of the input
 * is decoded by one batched launch (its codec from the signal column's type; pgnano blobs with
 * `pgnano_variant`, PGN_VARIANT_C5 for the reference's default build), re-encoded by one batched
 * launch as `dst_signal_type` (PGN_POD5_SIGNAL_*), packed on the device, and written with
 * pgn_pod5_write_file(source = the input).  Rows above PGN_MAX_CHUNK_SAMPLES samples fail with
 * PGN_ERR_UNSUPPORTED; a row the codec refuses fails the call with its status (detail in
 * pgn_pod5_last_error, pgnano_pod5.h). */
int pgn_pod5_transcode_file(pgn_ctx *ctx, const char *in_path, const char *out_path, int dst_signal_type,
                            int pgnano_variant, uint32_t rows_per_batch, pgn_pod5_transcode_stats *stats);

/* pgn_pod5_transcode_file with flags: PGN_POD5_KEEP_GOING -- a row the encoder refuses does not fail
 * the call; the file is written as the reference's `copy` writes it after a failing read
 * (pgn_pod5_write_file_keep_going), the outcome in *keep_going (may be NULL).  Rows whose input
 * does not decode still fail the call (the reference's copy logs them and writes unspecified
 * signal). */
#define PGN_POD5_KEEP_GOING 1u
int pgn_pod5_transcode_file_ex(pgn_ctx *ctx, const char *in_path, const char *out_path, int dst_signal_type,
                               int pgnano_variant, uint32_t rows_per_batch, uint32_t flags,
                               pgn_pod5_transcode_stats *stats, pgn_pod5_keep_going_result *keep_going);

/* One rank's share of a multi-GPU `copy` (the reference's writer takes whole read batches,
 * c_api.cpp:1104-1110; its reader decodes record batches, signal_table_reader.cpp:294-318): the
 * signal column of record batches batch_ids[0 .. n) of `f`, in that order, transcoded on ctx's GPU
 * exactly as pgn_pod5_transcode_file does.  The ranks' parts, put back in record-batch order, are
 * the column pgn_pod5_transcode_file writes (the caller gathers them and writes the file with
 * pgn_pod5_write_file).  The result is owned by *out: pgn_pod5_part_get, then pgn_pod5_part_free. */
typedef struct pgn_pod5_part pgn_pod5_part;
int pgn_pod5_transcode_part(pgn_ctx *ctx, const pgn_pod5_file *f, const uint32_t *batch_ids, uint32_t n,
                            int dst_signal_type, int pgnano_variant, pgn_pod5_part **out,
                            pgn_pod5_transcode_stats *stats);
/* rows of the part; offsets: rows + 1 entries into data (offsets[0] = 0). Valid until part_free. */
int pgn_pod5_part_get(const pgn_pod5_part *part, uint64_t *rows, const uint64_t **offsets, const uint8_t **data);
int pgn_pod5_part_free(pgn_pod5_part *part);

#ifdef __cplusplus
}
#endif

#endif /* PGNANO_POD5FILE_H */
