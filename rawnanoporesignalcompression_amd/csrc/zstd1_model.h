// zstd1_model.h -- serial composition of zstd1_common.h into a full `ZSTD_compress(.., 1)` for one
// source (a single-segment frame up to 512 KiB, a window-descriptor frame above).
//
// Host and device: the GPU kernels run the serial parts of these on one lane; the host build
// (libpgn_model.so, test-only) lets the test-suite fuzz the exact same code against libzstd.
//
// Parts of this file restate algorithms of Zstandard (libzstd 1.4.x), Copyright (c) 2016-present,
// Facebook, Inc., used under its BSD licence: see THIRD_PARTY_NOTICES.md at the repository root.
#pragma once
#include "zstd1_common.h"

namespace pgn {
namespace z1 {

// ---------------------------------------------------------------------------------------------
// ZSTD_compressBlock_fast (libzstd 1.4.x, two positions per step, kSearchStrength 8, stepSize 2) over
// the block [start, end) of a frame: window base = src - 1 (table entries hold indices = offset + 1,
// and persist across the blocks of a frame; the caller zeroes the table once per frame).  A source
// within the window (single segment, n <= 2^windowLog) has prefixStartIndex 1; above it, the block's
// candidates must lie within 2^windowLog of the block's end (ZSTD_getLowestPrefixIndex).  rep[0..1] are the confirmed
// repeat offsets on entry and the block's candidates on exit (ZSTD_compressBlock_fast_generic's
// offsetSaved rule); at the first position of the frame, offset_2 (4) > maxRep (1) is invalidated.
// Appends sequences (literal runs are implied: src[anchor .. anchor + litLength)); returns nbSeq,
// *lastLL = trailing literal run of the block.
// ---------------------------------------------------------------------------------------------
PGN_HD size_t match_count(const uint8_t* src, size_t a, size_t b, size_t end)
{
    size_t n = 0;
    while (a + n < end && src[a + n] == src[b + n]) n++;
    return n;
}

PGN_HD size_t fast_search_serial(const uint8_t* src, size_t start, size_t end, const Params& p, uint32_t* ht,
                                 uint32_t rep[3], Seq* seqs, size_t* lastLL)
{
    const unsigned hlog = p.hashLog, mls = p.mls;
    size_t nbSeq = 0;
    long ip0 = (long)start + (start == 0 ? 1 : 0), anchor = (long)start;
    long ip1 = ip0 + 1;
    const long iend = (long)end, ilimit = (long)end - 8;
    // ZSTD_getLowestPrefixIndex: candidates must lie within the window of the block's end
    const uint32_t lowIdx = window_low_index(end, p.windowLog);
    const long prefixStart = (long)lowIdx - 1;  // its position
    uint32_t offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;
    {
        // current - windowLow at the first position
        const uint32_t maxRep = (uint32_t)ip0 + 1u - window_low_index((size_t)ip0, p.windowLog);
        if (offset_2 > maxRep) { offsetSaved = offset_2; offset_2 = 0; }
        if (offset_1 > maxRep) { offsetSaved = offset_1; offset_1 = 0; }
    }
    while (ip1 < ilimit) {
        long ip2 = ip0 + 2;
        uint32_t h0 = hash_at(src + ip0, hlog, mls);
        uint32_t h1 = hash_at(src + ip1, hlog, mls);
        uint32_t val0 = rd32(src + ip0), val1 = rd32(src + ip1);
        uint32_t cur0 = (uint32_t)ip0 + 1, cur1 = (uint32_t)ip1 + 1;
        uint32_t mi0 = ht[h0], mi1 = ht[h1];
        ht[h0] = cur0;
        ht[h1] = cur1;
        long match0;
        size_t mLength;
        uint32_t offcode;
        if ((offset_1 > 0) && (rd32(src + ip2 - offset_1) == rd32(src + ip2))) {
            mLength = (src[ip2 - 1] == src[ip2 - (long)offset_1 - 1]) ? 1 : 0;
            ip0 = ip2 - (long)mLength;
            match0 = ip0 - (long)offset_1;
            mLength += 4;
            offcode = 0;
        } else {
            bool found = false;
            if ((mi0 > lowIdx) && rd32(src + mi0 - 1) == val0) {
                match0 = (long)mi0 - 1;
                found = true;
            } else if ((mi1 > lowIdx) && rd32(src + mi1 - 1) == val1) {
                ip0 = ip1;
                match0 = (long)mi1 - 1;
                found = true;
            }
            if (!found) {
                long step = ((ip0 - anchor) >> 7) + 2;
                ip0 += step;
                ip1 += step;
                continue;
            }
            offset_2 = offset_1;
            offset_1 = (uint32_t)(ip0 - match0);
            offcode = offset_1 + 2;
            mLength = 4;
            while ((ip0 > anchor) && (match0 > prefixStart) && (src[ip0 - 1] == src[match0 - 1])) {
                ip0--;
                match0--;
                mLength++;
            }
        }
        mLength += match_count(src, (size_t)ip0 + mLength, (size_t)match0 + mLength, (size_t)iend);
        seqs[nbSeq].litLength = (uint32_t)(ip0 - anchor);
        seqs[nbSeq].offset = offcode + 1;
        seqs[nbSeq].mlBase = (uint32_t)(mLength - 3);
        nbSeq++;
        ip0 += (long)mLength;
        anchor = ip0;
        if (ip0 <= ilimit) {
            ht[hash_at(src + cur0 + 1, hlog, mls)] = cur0 + 2;
            ht[hash_at(src + ip0 - 2, hlog, mls)] = (uint32_t)(ip0 - 2) + 1;
            if (offset_2 > 0) {
                while ((ip0 <= ilimit) && (rd32(src + ip0) == rd32(src + ip0 - offset_2))) {
                    size_t rLength = match_count(src, (size_t)ip0 + 4, (size_t)ip0 + 4 - offset_2, (size_t)iend) + 4;
                    uint32_t t = offset_2; offset_2 = offset_1; offset_1 = t;
                    ht[hash_at(src + ip0, hlog, mls)] = (uint32_t)ip0 + 1;
                    ip0 += (long)rLength;
                    seqs[nbSeq].litLength = 0;
                    seqs[nbSeq].offset = 1;
                    seqs[nbSeq].mlBase = (uint32_t)(rLength - 3);
                    nbSeq++;
                    anchor = ip0;
                }
            }
        }
        ip1 = ip0 + 1;
    }
    rep[0] = offset_1 ? offset_1 : offsetSaved;
    rep[1] = offset_2 ? offset_2 : offsetSaved;
    *lastLL = (size_t)(iend - anchor);
    return nbSeq;
}

// ---------------------------------------------------------------------------------------------
// Literals section (ZSTD_compressLiterals -> HUF_compress{1,4}X_repeat).  `prev` is the Huffman
// table state the frame carries from its last compressed block (HUF_repeat_none on the first
// block; HUF_repeat_check once a table was built -- level 1 never reaches HUF_repeat_valid);
// `next` receives this block's state (confirmed by the caller only if the block is emitted
// compressed).  `work` must hold a LitWork.  Returns the section size written at dst.
// ---------------------------------------------------------------------------------------------
struct HufState {
    uint8_t nbBits[256];  // 0 for symbols the table does not hold
    uint16_t val[256];
    bool check;           // HUF_repeat_check: the table may be reused
};

struct LitWork {
    uint32_t count[256];
    HufNode nodes[2 * 256 + 1];
    uint8_t nbBits[256];
    uint16_t val[256];
    FseCTable fct;
    uint8_t scratch[64];
};

PGN_HD size_t write_raw_literals(uint8_t* dst, const uint8_t* lit, size_t n)
{
    size_t fl = write_rawrle_lit_header(dst, n, kSetBasic);
    for (size_t i = 0; i < n; i++) dst[fl + i] = lit[i];
    return fl + n;
}

// Huffman-encode `n` symbols (1X stream) into dst; returns bytes (end mark included).
PGN_HD size_t huf_encode_1x(uint8_t* dst, const uint8_t* src, size_t n, const uint8_t* nbBits, const uint16_t* val)
{
    BitW bw;
    bw_init(bw, dst);
    for (size_t i = n; i-- > 0;) bw_add(bw, val[src[i]], nbBits[src[i]]);
    return bw_close(bw, dst);
}

// HUF_compress{1,4}X_usingCTable: the streams (and the 4X jump table) at dst; returns their size
PGN_HD size_t huf_encode_streams(uint8_t* dst, const uint8_t* lit, size_t n, bool singleStream, const uint8_t* nbBits,
                                 const uint16_t* val)
{
    if (singleStream) return huf_encode_1x(dst, lit, n, nbBits, val);
    const size_t seg = (n + 3) / 4;
    uint8_t* jt = dst;
    uint8_t* sp = jt + 6;
    for (int k = 0; k < 4; k++) {
        size_t a = seg * (size_t)k, b = (k == 3) ? n : seg * (size_t)(k + 1);
        size_t c = huf_encode_1x(sp, lit + a, b - a, nbBits, val);
        if (k < 3) wr16(jt + 2 * k, (uint32_t)c);
        sp += c;
    }
    return (size_t)(sp - dst);
}

// HUF_estimateCompressedSize
PGN_HD size_t huf_estimate(const uint8_t* nbBits, const uint32_t* count, unsigned maxSym)
{
    size_t bits = 0;
    for (unsigned s = 0; s <= maxSym; s++) bits += (size_t)nbBits[s] * count[s];
    return bits >> 3;
}

PGN_HD size_t compress_literals(uint8_t* dst, const uint8_t* lit, size_t n, LitWork& w, const HufState& prev,
                                HufState& next)
{
    next = prev;  // "Prepare nextEntropy assuming reusing the existing table"
    if (n <= 63) return write_raw_literals(dst, lit, n);
    const size_t minGain = (n >> 6) + 2;
    const size_t lhSize = huf_lit_header_size(n);
    const bool singleStream = n < 256;
    const bool preferRepeat = n <= 1024;  // strategy < ZSTD_lazy
    // HIST_count_wksp
    for (int s = 0; s < 256; s++) w.count[s] = 0;
    for (size_t i = 0; i < n; i++) w.count[lit[i]]++;
    unsigned maxSym = 255;
    while (w.count[maxSym] == 0) maxSym--;
    uint32_t largest = 0;
    for (unsigned s = 0; s <= maxSym; s++) if (w.count[s] > largest) largest = w.count[s];
    if (largest == n) {  // single symbol: RLE literals block
        size_t fl = write_rawrle_lit_header(dst, n, kSetRle);
        dst[fl] = lit[0];
        return fl + 1;
    }
    if (largest <= (n >> 7) + 4) return write_raw_literals(dst, lit, n);
    // HUF_validateCTable: the previous table must code every symbol present
    bool repeat = prev.check;
    if (repeat)
        for (unsigned s = 0; s <= maxSym; s++) repeat = repeat && !(w.count[s] != 0 && prev.nbBits[s] == 0);
    uint8_t* op = dst + lhSize;
    bool useOld = repeat && preferRepeat;
    size_t hSize = 0;
    if (!useOld) {
        unsigned huffLog = huf_optimal_table_log(kHufTableLogDefault, n, maxSym);
        for (int i = 0; i < 2 * 256 + 1; i++) { w.nodes[i].count = 0; w.nodes[i].parent = 0; w.nodes[i].byte = 0; w.nodes[i].nbBits = 0; }
        huf_sort_serial(w.nodes + 1, w.count, maxSym);
        huffLog = huf_build_from_sorted(w.nodes, maxSym, huffLog, w.nbBits, w.val);
        for (unsigned s = maxSym + 1; s < 256; s++) { w.nbBits[s] = 0; w.val[s] = 0; }
        hSize = huf_write_ctable(op, w.nbBits, maxSym, huffLog, w.fct, w.scratch);
        if (hSize == 0) return write_raw_literals(dst, lit, n);  // HUF_writeCTable error -> raw
        if (repeat) {  // is the previous table still the better one?
            const size_t oldSize = huf_estimate(prev.nbBits, w.count, maxSym);
            const size_t newSize = huf_estimate(w.nbBits, w.count, maxSym);
            if (oldSize <= hSize + newSize || hSize + 12 >= n) useOld = true;
        }
        if (!useOld && hSize + 12 >= n) return write_raw_literals(dst, lit, n);
    }
    size_t total;
    if (useOld) {  // HUF_compressCTable_internal with the previous table: no description
        const size_t c = huf_encode_streams(op, lit, n, singleStream, prev.nbBits, prev.val);
        if (c >= n - 1 || c >= n - minGain) return write_raw_literals(dst, lit, n);
        write_huf_lit_header(dst, lhSize, n, c, singleStream, kSetRepeat);
        return lhSize + c;
    }
    const size_t c = huf_encode_streams(op + hSize, lit, n, singleStream, w.nbBits, w.val);
    total = hSize + c;
    if (total >= n - 1) return write_raw_literals(dst, lit, n);        // HUF_compressCTable_internal
    if (total >= n - minGain) return write_raw_literals(dst, lit, n);  // ZSTD_compressLiterals
    write_huf_lit_header(dst, lhSize, n, total, singleStream);
    for (int s = 0; s < 256; s++) { next.nbBits[s] = w.nbBits[s]; next.val[s] = w.val[s]; }
    next.check = true;  // a newly built table: HUF_repeat_check
    return lhSize + total;
}

// ---------------------------------------------------------------------------------------------
// Sequences section (ZSTD_compressSequences_internal, repeat mode none).  Returns bytes written,
// or (size_t)-1 for "emit a raw block" (the <= 1.3.4 decoder workaround).
// ---------------------------------------------------------------------------------------------
struct SeqWork {
    FseCTable ll, of, ml;
    uint8_t tableSymbol[512];
    uint32_t count[kMaxML + 1];
    int16_t norm[kMaxML + 1];
};

PGN_HD size_t build_seq_table(uint8_t* op, FseCTable& ct, unsigned type, uint32_t* count, unsigned max,
                              unsigned lastCode, size_t nbSeq, unsigned fseLog, unsigned defaultNormLog,
                              unsigned defaultMax, int kind, SeqWork& w)
{
    if (type == kSetRle) {
        fse_build_ctable_rle(ct, max);
        op[0] = (uint8_t)lastCode;  // codeTable[0]; all codes are equal
        return 1;
    }
    if (type == kSetBasic) {
        for (unsigned s = 0; s <= defaultMax; s++)
            w.norm[s] = kind == 0 ? ll_default_norm(s) : (kind == 1 ? of_default_norm(s) : ml_default_norm(s));
        fse_build_ctable(ct, w.norm, defaultMax, defaultNormLog, w.tableSymbol);
        return 0;
    }
    // compressed
    size_t nbSeq_1 = nbSeq;
    unsigned tableLog = fse_optimal_table_log(fseLog, nbSeq, max, 2);
    if (count[lastCode] > 1) { count[lastCode]--; nbSeq_1--; }
    if (!fse_normalize(w.norm, tableLog, count, nbSeq_1, max, nbSeq_1 >= 2048)) return (size_t)-2;
    size_t nc = fse_write_ncount(op, w.norm, max, tableLog);
    if (nc == 0) return (size_t)-2;
    fse_build_ctable(ct, w.norm, max, tableLog, w.tableSymbol);
    return nc;
}

// codes: ll/of/ml code per sequence (filled here)
PGN_HD size_t compress_sequences(uint8_t* dst, const Seq* seqs, size_t nbSeq, uint8_t* llC, uint8_t* ofC,
                                 uint8_t* mlC, SeqWork& w)
{
    uint8_t* op = dst;
    if (nbSeq < 128) {
        *op++ = (uint8_t)nbSeq;
    } else if (nbSeq < 0x7F00) {
        op[0] = (uint8_t)((nbSeq >> 8) + 0x80);
        op[1] = (uint8_t)nbSeq;
        op += 2;
    } else {
        op[0] = 0xFF;
        wr16(op + 1, (uint32_t)(nbSeq - 0x7F00));
        op += 3;
    }
    if (nbSeq == 0) return (size_t)(op - dst);
    uint8_t* seqHead = op++;
    for (size_t i = 0; i < nbSeq; i++) {
        llC[i] = (uint8_t)ll_code(seqs[i].litLength);
        ofC[i] = (uint8_t)highbit32(seqs[i].offset);
        mlC[i] = (uint8_t)ml_code(seqs[i].mlBase);
    }
    uint8_t* lastNCount = nullptr;
    unsigned types[3];
    FseCTable* cts[3] = {&w.ll, &w.of, &w.ml};
    const uint8_t* codes[3] = {llC, ofC, mlC};
    const unsigned maxes[3] = {kMaxLL, kMaxOff, kMaxML};
    const unsigned fseLogs[3] = {kLLFSELog, kOffFSELog, kMLFSELog};
    const unsigned normLogs[3] = {kLLDefaultNormLog, kOFDefaultNormLog, kMLDefaultNormLog};
    const unsigned defMax[3] = {kMaxLL, kDefaultMaxOff, kMaxML};
    for (int k = 0; k < 3; k++) {
        // HIST_countFast_wksp
        for (unsigned s = 0; s <= kMaxML; s++) w.count[s] = 0;
        for (size_t i = 0; i < nbSeq; i++) w.count[codes[k][i]]++;
        unsigned max = maxes[k];
        while (max > 0 && w.count[max] == 0) max--;
        uint32_t mostFrequent = 0;
        for (unsigned s = 0; s <= max; s++) if (w.count[s] > mostFrequent) mostFrequent = w.count[s];
        bool defaultAllowed = (k == 1) ? (max <= kDefaultMaxOff) : true;
        types[k] = select_encoding_type(mostFrequent, nbSeq, normLogs[k], defaultAllowed);
        size_t sz = build_seq_table(op, *cts[k], types[k], w.count, max, codes[k][nbSeq - 1], nbSeq, fseLogs[k],
                                    normLogs[k], defMax[k], k, w);
        if (sz == (size_t)-2) return (size_t)-2;
        if (types[k] == kSetCompressed) lastNCount = op;
        op += sz;
    }
    *seqHead = (uint8_t)((types[0] << 6) + (types[1] << 4) + (types[2] << 2));
    // ZSTD_encodeSequences (no long offsets: windowLog <= 17)
    BitW bw;
    bw_init(bw, op);
    FseState sLL, sOF, sML;
    const size_t last = nbSeq - 1;
    fse_init_state2(sML, w.ml, mlC[last]);
    fse_init_state2(sOF, w.of, ofC[last]);
    fse_init_state2(sLL, w.ll, llC[last]);
    bw_add(bw, seqs[last].litLength, ll_bits(llC[last]));
    bw_add(bw, seqs[last].mlBase, ml_bits(mlC[last]));
    bw_add(bw, seqs[last].offset, ofC[last]);
    for (size_t n = nbSeq - 1; n-- > 0;) {
        fse_encode(bw, sOF, w.of, ofC[n]);
        fse_encode(bw, sML, w.ml, mlC[n]);
        fse_encode(bw, sLL, w.ll, llC[n]);
        bw_add(bw, seqs[n].litLength, ll_bits(llC[n]));
        bw_add(bw, seqs[n].mlBase, ml_bits(mlC[n]));
        bw_add(bw, seqs[n].offset, ofC[n]);
    }
    fse_flush(bw, sML, w.ml);
    fse_flush(bw, sOF, w.of);
    fse_flush(bw, sLL, w.ll);
    size_t streamSize = bw_close(bw, op);
    op += streamSize;
    if (lastNCount && (op - lastNCount) < 4) return (size_t)-1;
    return (size_t)(op - dst);
}

// ---------------------------------------------------------------------------------------------
// Blocks + frame (ZSTD_compress_frameChunk / ZSTD_compressBlock_internal, libzstd 1.4.8/1.4.9).
// ---------------------------------------------------------------------------------------------
PGN_HD size_t write_empty_frame(uint8_t* dst)
{
    size_t h = write_frame_header(dst, 0, 10);
    wr24(dst + h, 1u + (kBtRaw << 1));
    return h + 3;
}
PGN_HD size_t write_raw_block_frame(uint8_t* dst, const uint8_t* src, size_t n)
{
    size_t h = write_frame_header(dst, n, 10);
    wr24(dst + h, (uint32_t)(1u + (kBtRaw << 1) + (n << 3)));
    for (size_t i = 0; i < n; i++) dst[h + 3 + i] = src[i];
    return h + 3 + n;
}

struct CompressWork {
    LitWork lit;
    SeqWork seq;
    HufState huf[2];  // confirmed (previous compressed block) and candidate (this block)
};

// ZSTD_isRLE
PGN_HD bool block_is_rle(const uint8_t* p, size_t n)
{
    for (size_t i = 1; i < n; i++)
        if (p[i] != p[0]) return false;
    return true;
}

// One block [start, start + bs) of a frame: its header and body at dst; returns bytes written.
// `rep` / `huf` are the frame's confirmed state, updated when the block is emitted compressed
// (ZSTD_confirmRepcodesAndEntropyTables).  Sequence FSE tables never repeat at level 1 (the
// repeat mode stays "check", never "valid"), so they carry no state.
PGN_HD size_t compress_block(uint8_t* dst, const uint8_t* src, size_t start, size_t bs, bool last, bool first,
                             const Params& p, uint32_t* ht, uint32_t rep[3], Seq* seqs, uint8_t* llC, uint8_t* ofC,
                             uint8_t* mlC, uint8_t* litbuf, CompressWork& w)
{
    const uint8_t* blk = src + start;
    size_t cSize = 0;  // 0: raw block, 1: RLE block, else compressed body size
    if (bs >= 7) {     // MIN_CBLOCK_SIZE + ZSTD_blockHeaderSize + 1: below it no compression is tried
        uint32_t nrep[3] = {rep[0], rep[1], rep[2]};
        size_t lastLL = 0;
        const size_t nbSeq = fast_search_serial(src, start, start + bs, p, ht, nrep, seqs, &lastLL);
        const uint8_t* lit = blk;
        size_t nLit = bs;
        if (nbSeq > 0) {
            size_t pos = start, o = 0;
            for (size_t i = 0; i < nbSeq; i++) {
                for (uint32_t k = 0; k < seqs[i].litLength; k++) litbuf[o++] = src[pos + k];
                pos += seqs[i].litLength + seqs[i].mlBase + 3;
            }
            for (size_t k = 0; k < lastLL; k++) litbuf[o++] = src[pos + k];
            lit = litbuf;
            nLit = o;
        }
        uint8_t* body = dst + 3;
        const size_t litSize = compress_literals(body, lit, nLit, w.lit, w.huf[0], w.huf[1]);
        const size_t seqSize = compress_sequences(body + litSize, seqs, nbSeq, llC, ofC, mlC, w.seq);
        const size_t maxCSize = bs - ((bs >> 6) + 2);
        if (seqSize != (size_t)-1 && seqSize != (size_t)-2 && litSize + seqSize < maxCSize) cSize = litSize + seqSize;
        // a later block of one repeated byte is an RLE block (never the first: decoders <= 1.4.3)
        if (!first && cSize < 25 && block_is_rle(blk, bs)) cSize = 1;
        if (cSize > 1) {  // ZSTD_confirmRepcodesAndEntropyTables
            rep[0] = nrep[0];
            rep[1] = nrep[1];
            rep[2] = nrep[2];
            w.huf[0] = w.huf[1];
        }
    }
    if (cSize == 0) {
        wr24(dst, (uint32_t)((last ? 1u : 0u) + (kBtRaw << 1) + (bs << 3)));
        for (size_t i = 0; i < bs; i++) dst[3 + i] = blk[i];
        return 3 + bs;
    }
    if (cSize == 1) {
        wr24(dst, (uint32_t)((last ? 1u : 0u) + (kBtRle << 1) + (bs << 3)));
        dst[3] = blk[0];
        return 4;
    }
    wr24(dst, (uint32_t)((last ? 1u : 0u) + (kBtCompressed << 1) + (cSize << 3)));
    return 3 + cSize;
}

// Full serial ZSTD_compress(dst, bound, src, n, 1) (blocks of 128 KiB; a window-descriptor frame
// above 2^windowLog = 512 KiB).
// `ht`: 2^15 entries; `seqs`, `llC/ofC/mlC`: kMaxSrc/4 + 2 entries; `litbuf`: kMaxSrc bytes
// (per block); dst capacity >= compress_bound(n).
PGN_HD size_t compress_serial(uint8_t* dst, const uint8_t* src, size_t n, uint32_t* ht, Seq* seqs, uint8_t* llC,
                              uint8_t* ofC, uint8_t* mlC, uint8_t* litbuf, CompressWork& w)
{
    if (n == 0) return write_empty_frame(dst);
    if (n < 7) return write_raw_block_frame(dst, src, n);
    const Params p = level1_params(n);
    for (size_t i = 0; i < ((size_t)1 << p.hashLog); i++) ht[i] = 0;
    uint32_t rep[3] = {1, 4, 8};
    w.huf[0].check = false;
    for (int s = 0; s < 256; s++) { w.huf[0].nbBits[s] = 0; w.huf[0].val[s] = 0; }
    size_t o = write_frame_header(dst, n, p.windowLog);
    for (size_t start = 0; start < n; start += kMaxSrc) {
        const size_t bs = (n - start < kMaxSrc) ? n - start : kMaxSrc;
        o += compress_block(dst + o, src, start, bs, start + bs == n, start == 0, p, ht, rep, seqs, llC, ofC, mlC, litbuf, w);
    }
    return o;
}

}  // namespace z1
}  // namespace pgn
