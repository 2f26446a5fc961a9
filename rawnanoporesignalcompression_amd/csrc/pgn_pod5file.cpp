// pgn_pod5file.cpp -- POD5 combined-file and signal-table I/O without Arrow (include/pgnano_pod5file.h).
//
// Host code only.  Three layers, each restating a published format the reference reads and writes
// through libraries (flatbuffers, Arrow C++):
//   * flatbuffers: a bounds-checked table/vector/string reader, and a forward builder (parents
//     before children, so every uoffset points forward as the format requires; scalars aligned to
//     their size in the buffer, vtables before their tables);
//   * Arrow IPC file format (Schema.fbs / Message.fbs / File.fbs, metadata version V5): "ARROW1"
//     magic, encapsulated messages (0xFFFFFFFF, metadata length, flatbuffer padded to 8, body),
//     footer with the schema and record-batch blocks -- read for any schema (buffer and field-node
//     counts per type, pre-order), written for the signal table's three columns
//     (signal_table_schema.cpp:15-42);
//   * the POD5 combined layout (pod5/docs/SPECIFICATION.md; footer.fbs; written as
//     internal/combined_file_utils.h:85-151 and file_writer.cpp:300-350 write it, read as
//     combined_file_utils.h:188-279 reads it).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/pgnano_pod5file.h"

namespace {

thread_local std::string g_err;

struct Pod5Error : std::runtime_error {
    int status;
    Pod5Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};
[[noreturn]] void corrupt(const std::string& m) { throw Pod5Error(PGN_ERR_CORRUPT, m); }
[[noreturn]] void unsupported(const std::string& m) { throw Pod5Error(PGN_ERR_UNSUPPORTED, m); }

// ---------------------------------------------------------------------------------------------
// flatbuffers reader
struct Bytes {
    const uint8_t* p = nullptr;
    size_t n = 0;
};

template <class T>
T rd(const Bytes& b, size_t off)
{
    if (off > b.n || b.n - off < sizeof(T)) corrupt("flatbuffer read out of bounds");
    T v;
    memcpy(&v, b.p + off, sizeof(T));
    return v;
}

struct FbTable {
    Bytes b;
    size_t pos = 0, vt = 0;
    uint16_t vtsize = 0;
};

FbTable fb_table_at(const Bytes& b, size_t pos)
{
    FbTable t;
    t.b = b;
    t.pos = pos;
    const int32_t so = rd<int32_t>(b, pos);
    const int64_t vt = (int64_t)pos - (int64_t)so;
    if (vt < 0 || (size_t)vt + 4 > b.n) corrupt("flatbuffer vtable out of bounds");
    t.vt = (size_t)vt;
    t.vtsize = rd<uint16_t>(b, t.vt);
    if (t.vtsize < 4 || (t.vtsize & 1) || t.vt + t.vtsize > b.n) corrupt("flatbuffer vtable malformed");
    const uint16_t tsize = rd<uint16_t>(b, t.vt + 2);
    if (pos + tsize > b.n) corrupt("flatbuffer table out of bounds");
    return t;
}

FbTable fb_root(const Bytes& b) { return fb_table_at(b, rd<uint32_t>(b, 0)); }

// absolute position of field `id`, 0 if absent
size_t fb_field(const FbTable& t, int id)
{
    const size_t e = 4 + 2 * (size_t)id;
    if (e + 2 > t.vtsize) return 0;
    const uint16_t o = rd<uint16_t>(t.b, t.vt + e);
    return o ? t.pos + o : 0;
}

template <class T>
T fb_scalar(const FbTable& t, int id, T def)
{
    const size_t f = fb_field(t, id);
    return f ? rd<T>(t.b, f) : def;
}

// position referenced by the uoffset at `at`
size_t fb_deref(const Bytes& b, size_t at)
{
    const uint64_t target = (uint64_t)at + rd<uint32_t>(b, at);
    if (target >= b.n) corrupt("flatbuffer offset out of bounds");
    return (size_t)target;
}

bool fb_has(const FbTable& t, int id) { return fb_field(t, id) != 0; }

FbTable fb_subtable(const FbTable& t, int id)
{
    const size_t f = fb_field(t, id);
    if (!f) corrupt("flatbuffer: missing table field");
    return fb_table_at(t.b, fb_deref(t.b, f));
}

std::string fb_string_at(const Bytes& b, size_t pos)
{
    const uint32_t len = rd<uint32_t>(b, pos);
    if ((uint64_t)pos + 4 + len > b.n) corrupt("flatbuffer string out of bounds");
    return std::string((const char*)b.p + pos + 4, len);
}

bool fb_string(const FbTable& t, int id, std::string& out)
{
    const size_t f = fb_field(t, id);
    if (!f) return false;
    out = fb_string_at(t.b, fb_deref(t.b, f));
    return true;
}

struct FbVec {
    Bytes b;
    size_t start = 0;  // first element
    uint32_t len = 0;
};

FbVec fb_vector(const FbTable& t, int id, size_t elem_size)
{
    FbVec v;
    v.b = t.b;
    const size_t f = fb_field(t, id);
    if (!f) return v;
    const size_t p = fb_deref(t.b, f);
    v.len = rd<uint32_t>(t.b, p);
    v.start = p + 4;
    if ((uint64_t)v.start + (uint64_t)v.len * elem_size > t.b.n) corrupt("flatbuffer vector out of bounds");
    return v;
}

FbTable fb_vec_table(const FbVec& v, uint32_t i) { return fb_table_at(v.b, fb_deref(v.b, v.start + 4 * (size_t)i)); }

// ---------------------------------------------------------------------------------------------
// flatbuffers builder (forward: a node's children are placed after it)
struct FbNode;
using FbNodeP = std::shared_ptr<FbNode>;

struct FbField {
    int id;
    int size;  // scalar size in bytes (1, 2, 4, 8); 0 = offset to `child`
    uint64_t value;
    FbNodeP child;
};

struct FbNode {
    enum Kind { TABLE, STRING, VEC_OFFSETS, VEC_STRUCTS } kind = TABLE;
    std::vector<FbField> fields;         // TABLE
    std::string str;                     // STRING
    std::vector<FbNodeP> elems;          // VEC_OFFSETS
    std::vector<uint8_t> structs;        // VEC_STRUCTS: packed elements
    uint32_t count = 0, struct_align = 8;
};

FbNodeP fb_new_table() { return std::make_shared<FbNode>(); }
FbNodeP fb_new_string(const std::string& s)
{
    auto n = std::make_shared<FbNode>();
    n->kind = FbNode::STRING;
    n->str = s;
    return n;
}
FbNodeP fb_new_vec(std::vector<FbNodeP> elems)
{
    auto n = std::make_shared<FbNode>();
    n->kind = FbNode::VEC_OFFSETS;
    n->elems = std::move(elems);
    return n;
}
FbNodeP fb_new_structs(const void* data, uint32_t count, size_t elem_size, uint32_t align)
{
    auto n = std::make_shared<FbNode>();
    n->kind = FbNode::VEC_STRUCTS;
    n->structs.assign((const uint8_t*)data, (const uint8_t*)data + count * elem_size);
    n->count = count;
    n->struct_align = align;
    return n;
}
void fb_add(const FbNodeP& t, int id, int size, uint64_t v) { t->fields.push_back({id, size, v, nullptr}); }
void fb_add(const FbNodeP& t, int id, const FbNodeP& child) { t->fields.push_back({id, 0, 0, child}); }

struct FbBuilder {
    std::vector<uint8_t> b;
    void align(size_t a)
    {
        while (b.size() % a) b.push_back(0);
    }
    void put(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
    template <class T>
    void put(T v)
    {
        put(&v, sizeof(T));
    }
    template <class T>
    void set(size_t at, T v)
    {
        memcpy(b.data() + at, &v, sizeof(T));
    }
    void patch(size_t at, size_t target) { set<uint32_t>(at, (uint32_t)(target - at)); }

    size_t write(const FbNodeP& n)
    {
        switch (n->kind) {
        case FbNode::STRING: {
            align(4);
            const size_t pos = b.size();
            put<uint32_t>((uint32_t)n->str.size());
            put(n->str.data(), n->str.size());
            b.push_back(0);
            return pos;
        }
        case FbNode::VEC_STRUCTS: {
            // the length word sits just below the first element, which is aligned to struct_align
            align(4);
            while ((b.size() + 4) % n->struct_align) put<uint32_t>(0);
            const size_t pos = b.size();
            put<uint32_t>(n->count);
            put(n->structs.data(), n->structs.size());
            return pos;
        }
        case FbNode::VEC_OFFSETS: {
            align(4);
            const size_t pos = b.size();
            put<uint32_t>((uint32_t)n->elems.size());
            const size_t first = b.size();
            for (size_t i = 0; i < n->elems.size(); i++) put<uint32_t>(0);
            for (size_t i = 0; i < n->elems.size(); i++) patch(first + 4 * i, write(n->elems[i]));
            return pos;
        }
        case FbNode::TABLE:
        default: {
            // layout: soffset, then fields by decreasing size (each aligned to its size; the table
            // starts 8-aligned so relative alignment is absolute)
            std::vector<size_t> order(n->fields.size());
            for (size_t i = 0; i < order.size(); i++) order[i] = i;
            auto fsize = [&](size_t i) { return n->fields[i].size ? n->fields[i].size : 4; };
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t c) { return fsize(a) > fsize(c); });
            std::vector<uint16_t> foff(n->fields.size());
            size_t off = 4;
            int maxid = -1;
            for (size_t k : order) {
                const size_t s = fsize(k);
                off = (off + s - 1) / s * s;
                foff[k] = (uint16_t)off;
                off += s;
                maxid = std::max(maxid, n->fields[k].id);
            }
            const size_t tsize = (off + 3) & ~(size_t)3;
            // vtable
            align(2);
            const size_t vt = b.size();
            const uint16_t vtsize = (uint16_t)(4 + 2 * (maxid + 1));
            put<uint16_t>(vtsize);
            put<uint16_t>((uint16_t)tsize);
            std::vector<uint16_t> slots(maxid + 1, 0);
            for (size_t k = 0; k < n->fields.size(); k++) slots[n->fields[k].id] = foff[k];
            for (uint16_t s : slots) put<uint16_t>(s);
            align(8);
            const size_t pos = b.size();
            b.resize(pos + tsize, 0);
            set<int32_t>(pos, (int32_t)(pos - vt));
            for (size_t k = 0; k < n->fields.size(); k++) {
                const FbField& f = n->fields[k];
                if (f.size) memcpy(b.data() + pos + foff[k], &f.value, f.size);  // little-endian host
            }
            for (size_t k = 0; k < n->fields.size(); k++)
                if (!n->fields[k].size) patch(pos + foff[k], write(n->fields[k].child));
            return pos;
        }
        }
    }

    // finished buffer: root uoffset at 0, then the tree; the size is a multiple of 8 as a
    // flatbuffers builder's is (the POD5 reader locates the footer by its unpadded length,
    // combined_file_utils.h:211-218, so the footer must need no padding)
    static std::vector<uint8_t> finish(const FbNodeP& root)
    {
        FbBuilder fb;
        fb.put<uint32_t>(0);
        fb.align(8);
        fb.patch(0, fb.write(root));
        fb.align(8);
        return std::move(fb.b);
    }
};

// ---------------------------------------------------------------------------------------------
// Arrow IPC (format/Schema.fbs, Message.fbs, File.fbs)
enum ArrowType : uint8_t {
    AT_NONE = 0, AT_Null = 1, AT_Int = 2, AT_FloatingPoint = 3, AT_Binary = 4, AT_Utf8 = 5, AT_Bool = 6,
    AT_Decimal = 7, AT_Date = 8, AT_Time = 9, AT_Timestamp = 10, AT_Interval = 11, AT_List = 12, AT_Struct = 13,
    AT_Union = 14, AT_FixedSizeBinary = 15, AT_FixedSizeList = 16, AT_Map = 17, AT_Duration = 18,
    AT_LargeBinary = 19, AT_LargeUtf8 = 20, AT_LargeList = 21
};
constexpr int16_t kMetadataV5 = 4;
constexpr uint8_t kHeaderSchema = 1, kHeaderRecordBatch = 3;
const char kArrowMagic[6] = {'A', 'R', 'R', 'O', 'W', '1'};

struct KV {
    std::string key, value;
};

struct ArrowField {
    std::string name;
    uint8_t type = AT_NONE;
    int32_t int_bits = 0;
    bool int_signed = false;
    int32_t byte_width = 0;
    int16_t fp_precision = 0;  // FloatingPoint: 0 half, 1 single, 2 double
    bool dictionary = false;
    int32_t dict_bits = 32;    // dictionary index width (DictionaryEncoding.indexType, default int32)
    std::string ext_name;
    std::vector<ArrowField> children;
};

std::vector<KV> parse_kv(const FbTable& t, int id)
{
    std::vector<KV> out;
    const FbVec v = fb_vector(t, id, 4);
    for (uint32_t i = 0; i < v.len; i++) {
        const FbTable kv = fb_vec_table(v, i);
        KV e;
        fb_string(kv, 0, e.key);
        fb_string(kv, 1, e.value);
        out.push_back(std::move(e));
    }
    return out;
}

ArrowField parse_field(const FbTable& f, int depth)
{
    if (depth > 32) corrupt("Arrow schema nested too deeply");
    ArrowField a;
    fb_string(f, 0, a.name);
    a.type = fb_scalar<uint8_t>(f, 2, AT_NONE);
    if (fb_has(f, 3)) {
        const FbTable ty = fb_subtable(f, 3);
        if (a.type == AT_Int) {
            a.int_bits = fb_scalar<int32_t>(ty, 0, 0);
            a.int_signed = fb_scalar<uint8_t>(ty, 1, 0) != 0;
        } else if (a.type == AT_FixedSizeBinary) {
            a.byte_width = fb_scalar<int32_t>(ty, 0, 0);
        } else if (a.type == AT_FloatingPoint) {
            a.fp_precision = fb_scalar<int16_t>(ty, 0, 0);
        }
    }
    a.dictionary = fb_has(f, 4);
    if (a.dictionary) {
        const FbTable de = fb_subtable(f, 4);
        if (fb_has(de, 1)) a.dict_bits = fb_scalar<int32_t>(fb_subtable(de, 1), 0, 32);
    }
    const FbVec ch = fb_vector(f, 5, 4);
    for (uint32_t i = 0; i < ch.len; i++) a.children.push_back(parse_field(fb_vec_table(ch, i), depth + 1));
    for (const KV& kv : parse_kv(f, 6))
        if (kv.key == "ARROW:extension:name") a.ext_name = kv.value;
    return a;
}

// buffers and field nodes the field occupies in a record batch body (pre-order)
void count_layout(const ArrowField& a, size_t& nodes, size_t& buffers)
{
    nodes += 1;
    if (a.dictionary) {  // the batch holds the indices
        buffers += 2;
        return;
    }
    switch (a.type) {
    case AT_Null: break;
    case AT_Int: case AT_FloatingPoint: case AT_Bool: case AT_Decimal: case AT_Date: case AT_Time:
    case AT_Timestamp: case AT_Interval: case AT_Duration: case AT_FixedSizeBinary: buffers += 2; break;
    case AT_Binary: case AT_Utf8: case AT_LargeBinary: case AT_LargeUtf8: buffers += 3; break;
    case AT_List: case AT_LargeList: case AT_Map: buffers += 2; break;
    case AT_Struct: case AT_FixedSizeList: buffers += 1; break;
    default: unsupported("Arrow type id " + std::to_string(a.type) + " in a signal table");
    }
    for (const ArrowField& c : a.children) count_layout(c, nodes, buffers);
}

struct Block {
    int64_t offset;
    int32_t meta_len;
    int32_t pad;
    int64_t body_len;
};
static_assert(sizeof(Block) == 24, "Block struct layout");

struct ArrowBuf {
    int64_t offset, length;
};

// ---------------------------------------------------------------------------------------------
// the signal table of an open file
struct SignalBatch {
    uint64_t rows;
    const uint8_t* read_ids;      // 16 x rows
    const uint32_t* samples;      // rows (may be unaligned in a foreign file: read with memcpy)
    const uint8_t* offsets;       // rows + 1 int64 (bytes, or int16 elements when uncompressed)
    const uint8_t* data;          // signal bytes
    uint64_t data_len;            // bytes addressable from `data`
};

}  // namespace

struct pgn_pod5_file {
    std::vector<uint8_t> raw;
    std::string file_identifier, software, pod5_version;
    struct Embedded {
        int64_t offset, length;
        int content_type;
    };
    std::vector<Embedded> embedded;
    int signal_index = -1;
    // signal table
    int signal_type = PGN_POD5_SIGNAL_UNCOMPRESSED;
    std::vector<KV> schema_metadata, footer_metadata;
    std::vector<SignalBatch> batches;
    uint64_t rows = 0, data_bytes = 0, total_samples = 0;
};

namespace {

const uint8_t kPod5Signature[8] = {0x8B, 'P', 'O', 'D', '\r', '\n', 0x1A, '\n'};

int64_t ld_i64(const uint8_t* p)
{
    int64_t v;
    memcpy(&v, p, 8);
    return v;
}

// Arrow IPC file embedded at [base, base + len) of the file: signal-table columns
void parse_signal_table(pgn_pod5_file& f, size_t base, size_t len)
{
    const uint8_t* a = f.raw.data() + base;
    if (len < 18 || memcmp(a, kArrowMagic, 6) || memcmp(a + len - 6, kArrowMagic, 6))
        corrupt("signal table is not an Arrow IPC file");
    int32_t flen;
    memcpy(&flen, a + len - 10, 4);
    if (flen <= 0 || (size_t)flen > len - 18) corrupt("Arrow footer length out of range");
    const Bytes footer{a + len - 10 - flen, (size_t)flen};
    const FbTable ft = fb_root(footer);
    const FbTable schema = fb_subtable(ft, 1);
    f.footer_metadata = parse_kv(ft, 4);
    f.schema_metadata = parse_kv(schema, 2);
    if (fb_scalar<int16_t>(schema, 0, 0) != 0) unsupported("big-endian Arrow file");
    std::vector<ArrowField> fields;
    const FbVec fv = fb_vector(schema, 1, 4);
    for (uint32_t i = 0; i < fv.len; i++) fields.push_back(parse_field(fb_vec_table(fv, i), 0));
    // read_signal_table_schema (signal_table_schema.cpp:45-80)
    int iRead = -1, iSignal = -1, iSamples = -1;
    for (size_t i = 0; i < fields.size(); i++) {
        if (fields[i].name == "read_id") iRead = (int)i;
        if (fields[i].name == "signal") iSignal = (int)i;
        if (fields[i].name == "samples") iSamples = (int)i;
    }
    if (iRead < 0 || fields[iRead].type != AT_FixedSizeBinary || fields[iRead].byte_width != 16 ||
        fields[iRead].dictionary)
        corrupt("signal table: no read_id fixed_size_binary(16) column");
    if (iSamples < 0 || fields[iSamples].type != AT_Int || fields[iSamples].int_bits != 32 ||
        fields[iSamples].int_signed || fields[iSamples].dictionary)
        corrupt("signal table: no samples uint32 column");
    if (iSignal < 0 || fields[iSignal].dictionary) corrupt("signal table: no signal column");
    const ArrowField& sig = fields[iSignal];
    if (sig.type == AT_LargeList) {
        if (sig.children.size() != 1 || sig.children[0].type != AT_Int || sig.children[0].int_bits != 16 ||
            !sig.children[0].int_signed)
            corrupt("Schema field 'signal' list value type is incorrect type");
        f.signal_type = PGN_POD5_SIGNAL_UNCOMPRESSED;
    } else if (sig.type == AT_LargeBinary && sig.ext_name == "minknow.vbz") {
        f.signal_type = PGN_POD5_SIGNAL_VBZ;
    } else if (sig.type == AT_LargeBinary && sig.ext_name == "pgnano.signal") {
        f.signal_type = PGN_POD5_SIGNAL_PGNANO;
    } else {
        corrupt("Schema field 'signal' is incorrect type");
    }
    // where each column's buffers sit in a batch
    size_t firstBuf[3] = {0, 0, 0}, firstNode[3] = {0, 0, 0}, nodes = 0, buffers = 0;
    const int cols[3] = {iRead, iSignal, iSamples};
    for (size_t i = 0; i < fields.size(); i++) {
        for (int c = 0; c < 3; c++)
            if ((int)i == cols[c]) {
                firstBuf[c] = buffers;
                firstNode[c] = nodes;
            }
        count_layout(fields[i], nodes, buffers);
    }
    const FbVec bv = fb_vector(ft, 3, sizeof(Block));
    for (uint32_t i = 0; i < bv.len; i++) {
        Block blk;
        memcpy(&blk, footer.p + bv.start + (size_t)i * sizeof(Block), sizeof(Block));
        // compared without sums, so that values near INT64_MAX cannot wrap past the checks
        if (blk.offset < 8 || blk.meta_len < 8 || blk.body_len < 0 || (uint64_t)blk.offset > len ||
            (uint64_t)blk.meta_len > len - (uint64_t)blk.offset ||
            (uint64_t)blk.body_len > len - (uint64_t)blk.offset - (uint64_t)blk.meta_len)
            corrupt("Arrow record batch block out of range");
        const uint8_t* m = a + blk.offset;
        uint32_t cont;
        int32_t mlen;
        memcpy(&cont, m, 4);
        size_t hdr = 4;
        if (cont == 0xFFFFFFFFu) {
            memcpy(&mlen, m + 4, 4);
            hdr = 8;
        } else {
            mlen = (int32_t)cont;  // pre-0.15 framing
        }
        if (mlen <= 0 || (int64_t)hdr + mlen > blk.meta_len) corrupt("Arrow message length out of range");
        const Bytes mb{m + hdr, (size_t)mlen};
        const FbTable msg = fb_root(mb);
        if (fb_scalar<uint8_t>(msg, 1, 0) != kHeaderRecordBatch) corrupt("Arrow block is not a record batch");
        const FbTable rb = fb_subtable(msg, 2);
        if (fb_has(rb, 3)) unsupported("body-compressed signal table batches");
        const int64_t length = fb_scalar<int64_t>(rb, 0, 0);
        const FbVec nv = fb_vector(rb, 1, 16), bufv = fb_vector(rb, 2, 16);
        if (nv.len != nodes || bufv.len != buffers) corrupt("Arrow record batch layout does not match the schema");
        const uint8_t* body = a + blk.offset + blk.meta_len;
        auto node = [&](size_t k) {
            int64_t v[2];
            memcpy(v, mb.p + nv.start + 16 * k, 16);
            return std::make_pair(v[0], v[1]);
        };
        auto buf = [&](size_t k, int64_t need) {
            ArrowBuf bb;
            memcpy(&bb, mb.p + bufv.start + 16 * k, 16);
            if (bb.offset < 0 || bb.length < 0 || bb.offset > blk.body_len || bb.length > blk.body_len - bb.offset ||
                bb.length < need)
                corrupt("Arrow buffer out of range");
            return std::make_pair(body + bb.offset, bb.length);
        };
        // 16 bytes of read id per row: any larger length cannot fit the body (and 16 * length
        // below cannot overflow)
        if (length < 0 || length > blk.body_len / 16) corrupt("batch length out of range");
        for (int c = 0; c < 3; c++) {
            const auto nd = node(firstNode[c]);
            if (nd.first != length) corrupt("Arrow field length differs from the batch length");
            if (nd.second != 0) unsupported("null entries in a signal table column");
        }
        SignalBatch sb;
        sb.rows = (uint64_t)length;
        sb.read_ids = buf(firstBuf[0] + 1, 16 * length).first;
        sb.samples = (const uint32_t*)buf(firstBuf[2] + 1, 4 * length).first;
        sb.offsets = buf(firstBuf[1] + 1, 8 * (length + 1)).first;
        uint64_t first = (uint64_t)ld_i64(sb.offsets), last = (uint64_t)ld_i64(sb.offsets + 8 * length);
        if (f.signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED) {
            if (node(firstNode[1] + 1).second != 0) unsupported("null samples in an uncompressed signal column");
            const auto vals = buf(firstBuf[1] + 3, 0);  // child: validity, values
            sb.data = vals.first;
            sb.data_len = (uint64_t)vals.second;
            first *= 2;
            last *= 2;
        } else {
            const auto d = buf(firstBuf[1] + 2, 0);
            sb.data = d.first;
            sb.data_len = (uint64_t)d.second;
        }
        for (int64_t r = 0; r < length; r++)
            if (ld_i64(sb.offsets + 8 * r + 8) < ld_i64(sb.offsets + 8 * r)) corrupt("signal offsets not monotonic");
        if (last < first || last > sb.data_len) corrupt("signal offsets beyond the data buffer");
        f.batches.push_back(sb);
        f.rows += sb.rows;
        f.data_bytes += last - first;
        for (int64_t r = 0; r < length; r++) {
            uint32_t s;
            memcpy(&s, (const uint8_t*)sb.samples + 4 * r, 4);
            f.total_samples += s;
        }
    }
}

void parse_file(pgn_pod5_file& f)
{
    const std::vector<uint8_t>& r = f.raw;
    const size_t n = r.size();
    // combined_file_utils.h:192-221
    if (n < 8 + 16 + 8 + 8 + 16 + 8 || memcmp(r.data(), kPod5Signature, 8) || memcmp(r.data() + n - 8, kPod5Signature, 8))
        corrupt("Invalid signature in file");
    const size_t lenEnd = n - 8 - 16;
    const int64_t flen = ld_i64(r.data() + lenEnd - 8);
    if (flen < 0 || (uint64_t)flen > lenEnd - 8) corrupt("Invalid footer length");
    const Bytes fb{r.data() + lenEnd - 8 - flen, (size_t)flen};
    const FbTable ft = fb_root(fb);
    if (!fb_string(ft, 0, f.file_identifier)) corrupt("Invalid footer file_identifier");
    if (!fb_string(ft, 1, f.software)) corrupt("Invalid footer software");
    if (!fb_string(ft, 2, f.pod5_version)) corrupt("Invalid footer pod5_version");
    if (!fb_has(ft, 3)) corrupt("Invalid footer contents");
    const FbVec cv = fb_vector(ft, 3, 4);
    for (uint32_t i = 0; i < cv.len; i++) {
        const FbTable e = fb_vec_table(cv, i);
        pgn_pod5_file::Embedded em;
        em.offset = fb_scalar<int64_t>(e, 0, 0);
        em.length = fb_scalar<int64_t>(e, 1, 0);
        if (fb_scalar<int16_t>(e, 2, 0) != 0) corrupt("Invalid embedded file format");
        em.content_type = fb_scalar<int16_t>(e, 3, 0);
        if (em.content_type < 0 || em.content_type > PGN_POD5_CONTENT_RUN_INFO) corrupt("Unknown embedded file type");
        // open_sub_file (combined_file_utils.h:359-375)
        if (em.length < 0 || em.offset < 0 || (uint64_t)em.length > n || (uint64_t)em.offset > n - (uint64_t)em.length)
            corrupt("Bad footer info");
        if (em.content_type == PGN_POD5_CONTENT_SIGNAL) f.signal_index = (int)f.embedded.size();
        f.embedded.push_back(em);
    }
    if (f.signal_index < 0) corrupt("no signal table in the footer");
    const auto& s = f.embedded[f.signal_index];
    parse_signal_table(f, (size_t)s.offset, (size_t)s.length);
}

// ---------------------------------------------------------------------------------------------
// writer
FbNodeP kv_vec(const std::vector<KV>& kvs)
{
    std::vector<FbNodeP> v;
    for (const KV& kv : kvs) {
        auto t = fb_new_table();
        fb_add(t, 0, fb_new_string(kv.key));
        fb_add(t, 1, fb_new_string(kv.value));
        v.push_back(t);
    }
    return fb_new_vec(v);
}

FbNodeP field_node(const std::string& name, uint8_t type, FbNodeP type_table, std::vector<FbNodeP> children,
                   const std::vector<KV>& md)
{
    auto f = fb_new_table();
    fb_add(f, 0, fb_new_string(name));
    fb_add(f, 1, 1, 1);  // nullable (arrow::field default)
    fb_add(f, 2, 1, type);
    fb_add(f, 3, type_table);
    fb_add(f, 5, fb_new_vec(std::move(children)));
    if (!md.empty()) fb_add(f, 6, kv_vec(md));
    return f;
}

FbNodeP int_type(int bits, bool is_signed)
{
    auto t = fb_new_table();
    fb_add(t, 0, 4, (uint64_t)(uint32_t)bits);
    fb_add(t, 1, 1, is_signed ? 1 : 0);
    return t;
}

// make_signal_table_schema (signal_table_schema.cpp:10-42)
FbNodeP signal_schema(int signal_type, const std::vector<KV>& metadata)
{
    auto fsb = fb_new_table();
    fb_add(fsb, 0, 4, 16);
    std::vector<FbNodeP> fields;
    fields.push_back(field_node("read_id", AT_FixedSizeBinary, fsb, {},
                                {{"ARROW:extension:name", "minknow.uuid"}, {"ARROW:extension:metadata", ""}}));
    if (signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED) {
        auto item = field_node("item", AT_Int, int_type(16, true), {}, {});
        fields.push_back(field_node("signal", AT_LargeList, fb_new_table(), {item}, {}));
    } else {
        const char* ext = signal_type == PGN_POD5_SIGNAL_VBZ ? "minknow.vbz" : "pgnano.signal";
        fields.push_back(field_node("signal", AT_LargeBinary, fb_new_table(), {},
                                    {{"ARROW:extension:name", ext}, {"ARROW:extension:metadata", ""}}));
    }
    fields.push_back(field_node("samples", AT_Int, int_type(32, false), {}, {}));
    auto s = fb_new_table();
    fb_add(s, 0, 2, 0);  // little endian
    fb_add(s, 1, fb_new_vec(fields));
    if (!metadata.empty()) fb_add(s, 2, kv_vec(metadata));
    return s;
}

FbNodeP message(uint8_t header_type, FbNodeP header, int64_t body_len)
{
    auto m = fb_new_table();
    fb_add(m, 0, 2, (uint64_t)(uint16_t)kMetadataV5);
    fb_add(m, 1, 1, header_type);
    fb_add(m, 2, header);
    fb_add(m, 3, 8, (uint64_t)body_len);
    return m;
}

struct Out {
    std::vector<uint8_t> b;
    void put(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
    void pad(size_t a)
    {
        while (b.size() % a) b.push_back(0);
    }
};

// encapsulated message: 0xFFFFFFFF, metadata length (flatbuffer padded so that the body is 8-aligned)
int32_t put_message(Out& o, const std::vector<uint8_t>& fbm)
{
    const uint32_t cont = 0xFFFFFFFFu;
    const int32_t padded = (int32_t)((fbm.size() + 7) & ~(size_t)7);
    o.put(&cont, 4);
    o.put(&padded, 4);
    o.put(fbm.data(), fbm.size());
    o.b.resize(o.b.size() + (padded - fbm.size()), 0);
    return padded + 8;
}

// the signal table as an Arrow IPC file (MakeFileWriter + write_batch every rows_per_batch rows,
// signal_table_writer.cpp:280-330,404-450)
// data == nullptr: the signal bytes are left zero (reserved for positioned writes); positions (may be
// null) receives, per row, the table-relative offset of the row's signal bytes.
std::vector<uint8_t> write_signal_table(int signal_type, uint64_t rows, const uint8_t* read_ids, const uint32_t* samples,
                                        const uint64_t* offsets, const uint8_t* data, uint32_t rows_per_batch,
                                        const std::vector<KV>& schema_md, const std::vector<KV>& footer_md,
                                        uint64_t* positions = nullptr)
{
    Out o;
    o.put(kArrowMagic, 6);
    o.pad(8);
    put_message(o, FbBuilder::finish(message(kHeaderSchema, signal_schema(signal_type, schema_md), 0)));
    std::vector<Block> blocks;
    const bool unc = signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED;
    for (uint64_t r0 = 0; r0 < rows; r0 += rows_per_batch) {
        const uint64_t nr = std::min<uint64_t>(rows_per_batch, rows - r0);
        const uint64_t d0 = offsets[r0], d1 = offsets[r0 + nr];
        // body buffers, each padded to 8: read_id (validity, values), signal (validity, offsets,
        // data | child validity, child values), samples (validity, values)
        std::vector<int64_t> offs(nr + 1);
        for (uint64_t i = 0; i <= nr; i++) offs[i] = (int64_t)(offsets[r0 + i] - d0) / (unc ? 2 : 1);
        struct Piece {
            const void* p;
            int64_t n;
        };
        std::vector<Piece> pieces = {{nullptr, 0}, {read_ids + 16 * r0, (int64_t)(16 * nr)}, {nullptr, 0},
                                     {offs.data(), (int64_t)(8 * (nr + 1))}};
        if (unc) pieces.push_back({nullptr, 0});
        const size_t dataPiece = pieces.size();
        pieces.push_back({data ? data + d0 : nullptr, (int64_t)(d1 - d0)});
        pieces.push_back({nullptr, 0});
        pieces.push_back({samples + r0, (int64_t)(4 * nr)});
        std::vector<ArrowBuf> bufs;
        int64_t at = 0;
        for (const Piece& p : pieces) {
            bufs.push_back({at, p.n});
            at += (p.n + 7) & ~(int64_t)7;
        }
        std::vector<int64_t> nodes = {(int64_t)nr, 0, (int64_t)nr, 0};
        if (unc) {
            nodes.push_back(offs[nr]);
            nodes.push_back(0);
        }
        nodes.push_back((int64_t)nr);
        nodes.push_back(0);
        auto rb = fb_new_table();
        fb_add(rb, 0, 8, nr);
        fb_add(rb, 1, fb_new_structs(nodes.data(), (uint32_t)(nodes.size() / 2), 16, 8));
        fb_add(rb, 2, fb_new_structs(bufs.data(), (uint32_t)bufs.size(), 16, 8));
        Block blk;
        blk.offset = (int64_t)o.b.size();
        blk.meta_len = put_message(o, FbBuilder::finish(message(kHeaderRecordBatch, rb, at)));
        blk.pad = 0;
        blk.body_len = at;
        for (size_t k = 0; k < pieces.size(); k++) {
            const Piece& p = pieces[k];
            if (k == dataPiece && positions)
                for (uint64_t i = 0; i < nr; i++) positions[r0 + i] = (uint64_t)o.b.size() + (offsets[r0 + i] - d0);
            if (p.n && p.p) o.put(p.p, (size_t)p.n);
            else if (p.n) o.b.resize(o.b.size() + (size_t)p.n, 0);
            o.pad(8);
        }
        blocks.push_back(blk);
    }
    const uint32_t eos[2] = {0xFFFFFFFFu, 0};
    o.put(eos, 8);
    auto ft = fb_new_table();
    fb_add(ft, 0, 2, (uint64_t)(uint16_t)kMetadataV5);
    fb_add(ft, 1, signal_schema(signal_type, schema_md));
    fb_add(ft, 2, fb_new_structs(nullptr, 0, sizeof(Block), 8));
    fb_add(ft, 3, fb_new_structs(blocks.data(), (uint32_t)blocks.size(), sizeof(Block), 8));
    if (!footer_md.empty()) fb_add(ft, 4, kv_vec(footer_md));
    const std::vector<uint8_t> fbf = FbBuilder::finish(ft);
    o.put(fbf.data(), fbf.size());
    const int32_t fl = (int32_t)fbf.size();
    o.put(&fl, 4);
    o.put(kArrowMagic, 6);
    return std::move(o.b);
}

// ---------------------------------------------------------------------------------------------
// Row filter over an Arrow IPC file: the reads table of a keep-going copy (the reads the reference's
// `copy` writes when a read batch fails part-way, src/c++/copy.cpp:174-176, c_api.cpp:1118-1127).
// The schema message, the dictionary batches and the footer are copied byte for byte (the footer's
// block offsets and lengths patched in place); every record batch is rewritten with its kept rows,
// and the values of the list column `signal` (signal-table row indices) are renumbered.
struct IpcBatchIn {
    const uint8_t* body;
    int64_t bodyLen;
    Bytes meta;
    size_t nodes, bufs;  // vector starts in meta
    uint32_t nNodes, nBufs;
    uint32_t ni = 0, bi = 0;
    std::pair<int64_t, int64_t> node()
    {
        if (ni >= nNodes) corrupt("Arrow record batch has fewer field nodes than its schema");
        int64_t v[2];
        memcpy(v, meta.p + nodes + 16 * (size_t)ni++, 16);
        return {v[0], v[1]};
    }
    std::pair<const uint8_t*, int64_t> buf()
    {
        if (bi >= nBufs) corrupt("Arrow record batch has fewer buffers than its schema");
        ArrowBuf b;
        memcpy(&b, meta.p + bufs + 16 * (size_t)bi++, 16);
        if (b.offset < 0 || b.length < 0 || b.offset > bodyLen || b.length > bodyLen - b.offset)
            corrupt("Arrow buffer out of range");
        return {body + b.offset, b.length};
    }
};
struct IpcBatchOut {
    std::vector<int64_t> nodes;
    std::vector<ArrowBuf> bufs;
    Out body;
    void put(const void* p, size_t n)
    {
        bufs.push_back({(int64_t)body.b.size(), (int64_t)n});
        if (n) body.put(p, n);
        body.pad(8);
    }
};

int fixed_width(const ArrowField& f)
{
    if (f.dictionary) return f.dict_bits / 8;
    switch (f.type) {
    case AT_Int: return f.int_bits / 8;
    case AT_FloatingPoint: return f.fp_precision == 0 ? 2 : (f.fp_precision == 1 ? 4 : 8);
    case AT_FixedSizeBinary: return f.byte_width;
    default: return 0;
    }
}

bool bit_at(const uint8_t* b, int64_t i) { return (b[i >> 3] >> (i & 7)) & 1; }

// the field's arrays for rows `rows` (ascending) of the input; `remap` renumbers a list's uint64 values
void filter_field(const ArrowField& f, IpcBatchIn& in, const std::vector<int64_t>& rows, IpcBatchOut& out,
                  const std::vector<int64_t>* remap)
{
    const auto nd = in.node();
    const int64_t L = nd.first, nulls = nd.second;
    if (L < 0 || nulls < 0) corrupt("Arrow field node out of range");
    for (int64_t r : rows)
        if (r >= L) corrupt("row beyond the Arrow array");
    const int64_t n = (int64_t)rows.size();
    if (f.type == AT_Null && !f.dictionary) {
        out.nodes.push_back(n);
        out.nodes.push_back(n);
        return;
    }
    // validity
    const auto vb = in.buf();
    int64_t newNulls = 0;
    std::vector<uint8_t> valid;
    if (nulls > 0) {
        if (vb.second * 8 < L) corrupt("Arrow validity bitmap too short");
        valid.assign((size_t)(n + 7) / 8, 0);
        for (int64_t i = 0; i < n; i++) {
            if (bit_at(vb.first, rows[i])) valid[i >> 3] |= (uint8_t)(1u << (i & 7));
            else newNulls++;
        }
    }
    out.nodes.push_back(n);
    out.nodes.push_back(newNulls);
    if (newNulls) out.put(valid.data(), valid.size());
    else out.put(nullptr, 0);
    const int w = fixed_width(f);
    if (w > 0) {
        const auto vals = in.buf();
        if (vals.second < L * w) corrupt("Arrow values buffer too short");
        std::vector<uint8_t> v((size_t)(n * w));
        for (int64_t i = 0; i < n; i++) memcpy(v.data() + i * w, vals.first + rows[i] * w, (size_t)w);
        out.put(v.data(), v.size());
        return;
    }
    switch (f.type) {
    case AT_Bool: {
        const auto vals = in.buf();
        if (vals.second * 8 < L) corrupt("Arrow bool buffer too short");
        std::vector<uint8_t> v((size_t)(n + 7) / 8, 0);
        for (int64_t i = 0; i < n; i++)
            if (bit_at(vals.first, rows[i])) v[i >> 3] |= (uint8_t)(1u << (i & 7));
        out.put(v.data(), v.size());
        return;
    }
    case AT_Binary: case AT_Utf8: case AT_LargeBinary: case AT_LargeUtf8:
    case AT_List: case AT_LargeList: {
        const bool large = f.type == AT_LargeBinary || f.type == AT_LargeUtf8 || f.type == AT_LargeList;
        const int ow = large ? 8 : 4;
        const auto ob = in.buf();
        if (ob.second < (L + 1) * ow) corrupt("Arrow offsets buffer too short");
        auto off = [&](int64_t i) -> int64_t {
            if (large) return ld_i64(ob.first + 8 * i);
            int32_t v;
            memcpy(&v, ob.first + 4 * i, 4);
            return v;
        };
        std::vector<uint8_t> no((size_t)((n + 1) * ow));
        std::vector<int64_t> child;
        int64_t at = 0;
        for (int64_t i = 0; i <= n; i++) {
            if (large) memcpy(no.data() + 8 * i, &at, 8);
            else {
                const int32_t v = (int32_t)at;
                memcpy(no.data() + 4 * i, &v, 4);
            }
            if (i == n) break;
            const int64_t a0 = off(rows[i]), a1 = off(rows[i] + 1);
            if (a0 < 0 || a1 < a0) corrupt("Arrow offsets not monotonic");
            for (int64_t k = a0; k < a1; k++) child.push_back(k);
            at += a1 - a0;
        }
        out.put(no.data(), no.size());
        if (f.type == AT_List || f.type == AT_LargeList) {
            if (f.children.size() != 1) corrupt("Arrow list without one child");
            filter_field(f.children[0], in, child, out, remap);
            if (remap) {  // renumber the child's values (uint64): the last buffer written
                const ArrowBuf& cb = out.bufs.back();
                for (int64_t i = 0; i < cb.length / 8; i++) {
                    uint64_t v;
                    memcpy(&v, out.body.b.data() + cb.offset + 8 * i, 8);
                    if (v >= remap->size() || (*remap)[v] < 0) corrupt("a kept read lists a dropped signal row");
                    const uint64_t nv = (uint64_t)(*remap)[v];
                    memcpy(out.body.b.data() + cb.offset + 8 * i, &nv, 8);
                }
            }
        } else {
            const auto db = in.buf();
            std::vector<uint8_t> d;
            for (int64_t i = 0; i < n; i++) {
                const int64_t a0 = off(rows[i]), a1 = off(rows[i] + 1);
                if (a1 > db.second) corrupt("Arrow data buffer too short");
                d.insert(d.end(), db.first + a0, db.first + a1);
            }
            out.put(d.data(), d.size());
        }
        return;
    }
    case AT_Struct:
        for (const ArrowField& c : f.children) filter_field(c, in, rows, out, nullptr);
        return;
    default:
        unsupported("Arrow type id " + std::to_string(f.type) + " in a table to filter");
    }
}

struct IpcReader {
    const uint8_t* a = nullptr;
    size_t len = 0;
    std::vector<ArrowField> fields;
    Bytes footer;
    FbVec dicts, batches;
    explicit IpcReader(const uint8_t* p, size_t n) : a(p), len(n)
    {
        if (len < 18 || memcmp(a, kArrowMagic, 6) || memcmp(a + len - 6, kArrowMagic, 6))
            corrupt("table is not an Arrow IPC file");
        int32_t flen;
        memcpy(&flen, a + len - 10, 4);
        if (flen <= 0 || (size_t)flen > len - 18) corrupt("Arrow footer length out of range");
        footer = Bytes{a + len - 10 - flen, (size_t)flen};
        const FbTable ft = fb_root(footer);
        const FbTable schema = fb_subtable(ft, 1);
        const FbVec fv = fb_vector(schema, 1, 4);
        for (uint32_t i = 0; i < fv.len; i++) fields.push_back(parse_field(fb_vec_table(fv, i), 0));
        dicts = fb_vector(ft, 2, sizeof(Block));
        batches = fb_vector(ft, 3, sizeof(Block));
    }
    Block block(const FbVec& v, uint32_t i) const
    {
        Block blk;
        memcpy(&blk, footer.p + v.start + (size_t)i * sizeof(Block), sizeof(Block));
        if (blk.offset < 8 || blk.meta_len < 8 || blk.body_len < 0 || (uint64_t)blk.offset > len ||
            (uint64_t)blk.meta_len > len - (uint64_t)blk.offset ||
            (uint64_t)blk.body_len > len - (uint64_t)blk.offset - (uint64_t)blk.meta_len)
            corrupt("Arrow block out of range");
        return blk;
    }
    IpcBatchIn batch(const Block& blk) const
    {
        const uint8_t* m = a + blk.offset;
        uint32_t cont;
        int32_t mlen;
        memcpy(&cont, m, 4);
        size_t hdr = 4;
        if (cont == 0xFFFFFFFFu) {
            memcpy(&mlen, m + 4, 4);
            hdr = 8;
        } else {
            mlen = (int32_t)cont;
        }
        if (mlen <= 0 || (int64_t)hdr + mlen > blk.meta_len) corrupt("Arrow message length out of range");
        IpcBatchIn in;
        in.meta = Bytes{m + hdr, (size_t)mlen};
        const FbTable msg = fb_root(in.meta);
        if (fb_scalar<uint8_t>(msg, 1, 0) != kHeaderRecordBatch) corrupt("Arrow block is not a record batch");
        const FbTable rb = fb_subtable(msg, 2);
        if (fb_has(rb, 3)) unsupported("body-compressed Arrow batches");
        const FbVec nv = fb_vector(rb, 1, 16), bv = fb_vector(rb, 2, 16);
        in.nodes = nv.start;
        in.nNodes = nv.len;
        in.bufs = bv.start;
        in.nBufs = bv.len;
        in.body = a + blk.offset + blk.meta_len;
        in.bodyLen = blk.body_len;
        return in;
    }
};

// the rows of record batch `blk` of the reads table and each read's signal rows
void read_signal_lists(const IpcReader& r, const Block& blk, int iSignal, std::vector<std::vector<int64_t>>& lists)
{
    IpcBatchIn in = r.batch(blk);
    lists.clear();
    for (int c = 0; c < (int)r.fields.size(); c++) {
        if (c != iSignal) {
            size_t nodes = 0, buffers = 0;
            count_layout(r.fields[c], nodes, buffers);
            in.ni += (uint32_t)nodes;
            in.bi += (uint32_t)buffers;
            continue;
        }
        const auto nd = in.node();
        const int64_t L = nd.first;
        (void)in.buf();  // validity
        const auto ob = in.buf();
        const ArrowField& f = r.fields[c];
        const bool large = f.type == AT_LargeList;
        if (L < 0 || ob.second < (L + 1) * (large ? 8 : 4)) corrupt("reads.signal offsets too short");
        (void)in.node();
        (void)in.buf();  // child validity
        const auto vb = in.buf();
        for (int64_t i = 0; i < L; i++) {
            int64_t a0, a1;
            if (large) {
                a0 = ld_i64(ob.first + 8 * i);
                a1 = ld_i64(ob.first + 8 * i + 8);
            } else {
                int32_t x, y;
                memcpy(&x, ob.first + 4 * i, 4);
                memcpy(&y, ob.first + 4 * i + 4, 4);
                a0 = x;
                a1 = y;
            }
            if (a0 < 0 || a1 < a0 || a1 * 8 > vb.second) corrupt("reads.signal offsets out of range");
            std::vector<int64_t> rowsOf;
            for (int64_t k = a0; k < a1; k++) rowsOf.push_back(ld_i64(vb.first + 8 * k));
            lists.push_back(std::move(rowsOf));
        }
        return;
    }
}

// The reads table with the reads keepRead[i] (reads in file order) and signal rows renumbered.
std::vector<uint8_t> filter_reads_table(const IpcReader& r, int iSignal, const std::vector<bool>& keepRead,
                                        const std::vector<int64_t>& remap)
{
    // messages in file order: dictionaries (copied) and record batches (rewritten)
    struct Item {
        Block blk;
        bool batch;
        uint32_t idx;
    };
    std::vector<Item> items;
    for (uint32_t i = 0; i < r.dicts.len; i++) items.push_back({r.block(r.dicts, i), false, i});
    for (uint32_t i = 0; i < r.batches.len; i++) items.push_back({r.block(r.batches, i), true, i});
    std::sort(items.begin(), items.end(), [](const Item& x, const Item& y) { return x.blk.offset < y.blk.offset; });
    const int64_t schemaEnd = items.empty() ? (int64_t)r.len - 10 - (int64_t)r.footer.n - 8 : items[0].blk.offset;
    Out o;
    o.put(r.a, (size_t)schemaEnd);  // magic and the schema message
    std::vector<Block> newDict(r.dicts.len), newBatch(r.batches.len);
    uint64_t read0 = 0;  // first read (file order) of the next record batch
    std::vector<Item> byIdx(items);
    std::sort(byIdx.begin(), byIdx.end(), [](const Item& x, const Item& y) {
        return x.batch != y.batch ? !x.batch : x.idx < y.idx;
    });
    std::vector<uint64_t> firstRead(r.batches.len, 0);
    for (const Item& it : byIdx)
        if (it.batch) {
            firstRead[it.idx] = read0;
            read0 += (uint64_t)std::max<int64_t>(0, r.batch(it.blk).node().first);
        }
    for (const Item& it : items) {
        if (!it.batch) {
            Block b = it.blk;
            b.offset = (int64_t)o.b.size();
            o.put(r.a + it.blk.offset, (size_t)(it.blk.meta_len + it.blk.body_len));
            newDict[it.idx] = b;
            continue;
        }
        IpcBatchIn in = r.batch(it.blk);
        const FbTable rb = fb_subtable(fb_root(in.meta), 2);
        const int64_t length = fb_scalar<int64_t>(rb, 0, 0);
        std::vector<int64_t> rows;
        for (int64_t i = 0; i < length; i++)
            if (keepRead.at(firstRead[it.idx] + (uint64_t)i)) rows.push_back(i);
        IpcBatchOut out;
        for (int c = 0; c < (int)r.fields.size(); c++) filter_field(r.fields[c], in, rows, out, c == iSignal ? &remap : nullptr);
        if (in.ni != in.nNodes || in.bi != in.nBufs) corrupt("Arrow record batch layout does not match the schema");
        auto rbo = fb_new_table();
        fb_add(rbo, 0, 8, (uint64_t)rows.size());
        fb_add(rbo, 1, fb_new_structs(out.nodes.data(), (uint32_t)(out.nodes.size() / 2), 16, 8));
        fb_add(rbo, 2, fb_new_structs(out.bufs.data(), (uint32_t)out.bufs.size(), 16, 8));
        Block b;
        b.offset = (int64_t)o.b.size();
        b.meta_len = put_message(o, FbBuilder::finish(message(kHeaderRecordBatch, rbo, (int64_t)out.body.b.size())));
        b.pad = 0;
        b.body_len = (int64_t)out.body.b.size();
        o.put(out.body.b.data(), out.body.b.size());
        newBatch[it.idx] = b;
    }
    const uint32_t eos[2] = {0xFFFFFFFFu, 0};
    o.put(eos, 8);
    // the footer, its blocks patched in place (same counts, fixed-size structs)
    std::vector<uint8_t> ftb(r.footer.p, r.footer.p + r.footer.n);
    for (uint32_t i = 0; i < r.dicts.len; i++) memcpy(ftb.data() + r.dicts.start + 24 * (size_t)i, &newDict[i], 24);
    for (uint32_t i = 0; i < r.batches.len; i++) memcpy(ftb.data() + r.batches.start + 24 * (size_t)i, &newBatch[i], 24);
    o.put(ftb.data(), ftb.size());
    const int32_t fl = (int32_t)ftb.size();
    o.put(&fl, 4);
    o.put(kArrowMagic, 6);
    return std::move(o.b);
}

std::string uuid_string(const uint8_t u[16])
{
    char s[40];
    snprintf(s, sizeof(s), "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", u[0], u[1], u[2],
             u[3], u[4], u[5], u[6], u[7], u[8], u[9], u[10], u[11], u[12], u[13], u[14], u[15]);
    return s;
}

void random_bytes(uint8_t* p, size_t n)
{
    std::random_device rd;
    for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rd();
}

std::vector<uint8_t> read_whole(const char* path)
{
    FILE* fp = fopen(path, "rb");
    if (!fp) throw Pod5Error(PGN_ERR_IO, std::string("cannot open ") + path);
    std::vector<uint8_t> v;
    if (fseek(fp, 0, SEEK_END) == 0) {
        const long sz = ftell(fp);
        if (sz > 0) {
            v.resize((size_t)sz);
            rewind(fp);
            if (fread(v.data(), 1, v.size(), fp) != v.size()) {
                fclose(fp);
                throw Pod5Error(PGN_ERR_IO, std::string("cannot read ") + path);
            }
        }
    }
    fclose(fp);
    return v;
}

template <class F>
int guarded(F&& fn)
{
    try {
        return fn();
    } catch (const Pod5Error& e) {
        g_err = e.what();
        return e.status;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return PGN_ERR_IO;
    } catch (const std::exception& e) {
        g_err = e.what();
        return PGN_ERR_CORRUPT;
    }
}

}  // namespace

extern "C" {

const char* pgn_pod5_file_error(void) { return g_err.c_str(); }

int pgn_pod5_file_open(const char* path, pgn_pod5_file** out)
{
    if (!path || !out) return PGN_ERR_INVALID_ARG;
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<pgn_pod5_file> f(new pgn_pod5_file());
        f->raw = read_whole(path);
        parse_file(*f);
        *out = f.release();
        return (int)PGN_OK;
    });
}

int pgn_pod5_file_close(pgn_pod5_file* f)
{
    if (!f) return PGN_ERR_INVALID_ARG;
    delete f;
    return PGN_OK;
}

const char* pgn_pod5_file_identifier(const pgn_pod5_file* f) { return f ? f->file_identifier.c_str() : nullptr; }
const char* pgn_pod5_file_software(const pgn_pod5_file* f) { return f ? f->software.c_str() : nullptr; }
const char* pgn_pod5_file_pod5_version(const pgn_pod5_file* f) { return f ? f->pod5_version.c_str() : nullptr; }

int pgn_pod5_file_embedded_count(const pgn_pod5_file* f) { return f ? (int)f->embedded.size() : 0; }

int pgn_pod5_file_embedded(const pgn_pod5_file* f, int index, int64_t* offset, int64_t* length, int* content_type)
{
    if (!f || index < 0 || index >= (int)f->embedded.size()) return PGN_ERR_INVALID_ARG;
    const auto& e = f->embedded[index];
    if (offset) *offset = e.offset;
    if (length) *length = e.length;
    if (content_type) *content_type = e.content_type;
    return PGN_OK;
}

int pgn_pod5_signal_info(const pgn_pod5_file* f, uint64_t* rows, uint32_t* batches, int* signal_type,
                         uint64_t* data_bytes, uint64_t* total_samples)
{
    if (!f) return PGN_ERR_INVALID_ARG;
    if (rows) *rows = f->rows;
    if (batches) *batches = (uint32_t)f->batches.size();
    if (signal_type) *signal_type = f->signal_type;
    if (data_bytes) *data_bytes = f->data_bytes;
    if (total_samples) *total_samples = f->total_samples;
    return PGN_OK;
}

int pgn_pod5_signal_read(const pgn_pod5_file* f, uint8_t* read_ids, uint32_t* samples, uint64_t* offsets, uint8_t* data)
{
    if (!f) return PGN_ERR_INVALID_ARG;
    const uint64_t scale = f->signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED ? 2 : 1;
    uint64_t row = 0, at = 0;
    if (offsets) offsets[0] = 0;
    for (const SignalBatch& b : f->batches) {
        if (read_ids) memcpy(read_ids + 16 * row, b.read_ids, 16 * b.rows);
        if (samples) memcpy(samples + row, b.samples, 4 * b.rows);
        const uint64_t first = (uint64_t)ld_i64(b.offsets) * scale;
        for (uint64_t r = 0; r < b.rows; r++) {
            const uint64_t end = (uint64_t)ld_i64(b.offsets + 8 * (r + 1)) * scale;
            if (offsets) offsets[row + r + 1] = at + end - first;
        }
        const uint64_t n = (uint64_t)ld_i64(b.offsets + 8 * b.rows) * scale - first;
        if (data && n) memcpy(data + at, b.data + first, n);
        at += n;
        row += b.rows;
    }
    return PGN_OK;
}

int pgn_pod5_signal_batch_rows(const pgn_pod5_file* f, uint32_t batch, uint64_t* first_row, uint64_t* rows)
{
    if (!f || batch >= f->batches.size()) return PGN_ERR_INVALID_ARG;
    uint64_t r0 = 0;
    for (uint32_t b = 0; b < batch; b++) r0 += f->batches[b].rows;
    if (first_row) *first_row = r0;
    if (rows) *rows = f->batches[batch].rows;
    return PGN_OK;
}

int pgn_pod5_signal_read_batches(const pgn_pod5_file* f, const uint32_t* batch_ids, uint32_t n, uint64_t* rows_out,
                                 uint64_t* data_bytes_out, uint64_t* samples_out, uint8_t* read_ids, uint32_t* samples,
                                 uint64_t* offsets, uint8_t* data)
{
    if (!f || (n && !batch_ids)) return PGN_ERR_INVALID_ARG;
    const uint64_t scale = f->signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED ? 2 : 1;
    uint64_t row = 0, at = 0, tot = 0;
    if (offsets) offsets[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (batch_ids[i] >= f->batches.size()) return PGN_ERR_INVALID_ARG;
        const SignalBatch& b = f->batches[batch_ids[i]];
        if (read_ids) memcpy(read_ids + 16 * row, b.read_ids, 16 * b.rows);
        if (samples) memcpy(samples + row, b.samples, 4 * b.rows);
        for (uint64_t r = 0; r < b.rows; r++) {
            uint32_t sm;
            memcpy(&sm, (const uint8_t*)b.samples + 4 * r, 4);
            tot += sm;
        }
        const uint64_t first = (uint64_t)ld_i64(b.offsets) * scale;
        for (uint64_t r = 0; r < b.rows; r++) {
            const uint64_t end = (uint64_t)ld_i64(b.offsets + 8 * (r + 1)) * scale;
            if (offsets) offsets[row + r + 1] = at + end - first;
        }
        const uint64_t m = (uint64_t)ld_i64(b.offsets + 8 * b.rows) * scale - first;
        if (data && m) memcpy(data + at, b.data + first, m);
        at += m;
        row += b.rows;
    }
    if (rows_out) *rows_out = row;
    if (data_bytes_out) *data_bytes_out = at;
    if (samples_out) *samples_out = tot;
    return PGN_OK;
}

int pgn_pod5_signal_batch_row_counts(const pgn_pod5_file* f, uint64_t* counts)
{
    if (!f || !counts) return PGN_ERR_INVALID_ARG;
    for (size_t b = 0; b < f->batches.size(); b++) counts[b] = f->batches[b].rows;
    return PGN_OK;
}

// pgn_pod5_write_file and pgn_pod5_write_file_reserved: data == nullptr leaves the signal bytes zero;
// positions (may be null) receives each row's file offset; write == false only computes positions.
static int write_file_impl(const char* path, const pgn_pod5_file* source, int signal_type, uint64_t rows,
                           const uint8_t* read_ids, const uint32_t* samples, const uint64_t* offsets,
                           const uint8_t* data, uint32_t rows_per_batch, const char* software,
                           const uint8_t* section_marker, bool write, uint64_t* positions,
                           const std::vector<uint8_t>* readsTable = nullptr)
{
    if ((write && !path) || (rows && (!read_ids || !samples || !offsets)) || signal_type < PGN_POD5_SIGNAL_UNCOMPRESSED ||
        signal_type > PGN_POD5_SIGNAL_PGNANO)
        return PGN_ERR_INVALID_ARG;
    for (uint64_t i = 0; i < rows; i++)
        if (offsets[i + 1] < offsets[i] ||
            (signal_type == PGN_POD5_SIGNAL_UNCOMPRESSED && (offsets[i + 1] - offsets[i]) != 2ull * samples[i]))
            return PGN_ERR_INVALID_ARG;
    if (rows_per_batch == 0) rows_per_batch = PGN_POD5_DEFAULT_SIGNAL_BATCH_ROWS;
    return guarded([&] {
        std::string ident, sw, ver;
        std::vector<KV> schema_md, footer_md;
        if (source) {
            ident = source->file_identifier;
            sw = source->software;
            ver = source->pod5_version;
            schema_md = source->schema_metadata;
            footer_md = source->footer_metadata;
        } else {
            uint8_t u[16];
            random_bytes(u, 16);
            u[6] = (uint8_t)((u[6] & 0x0F) | 0x40);  // version 4
            u[8] = (uint8_t)((u[8] & 0x3F) | 0x80);  // RFC 4122 variant
            ident = uuid_string(u);
            sw = software ? software : "rawnanoporesignalcompression_amd";
            ver = "0.3.10";
            schema_md = {{"MINKNOW:pod5_version", ver}, {"MINKNOW:software", sw}, {"MINKNOW:file_identifier", ident}};
            footer_md = schema_md;
        }
        uint8_t marker[16];
        if (section_marker)
            memcpy(marker, section_marker, 16);
        else
            random_bytes(marker, 16);
        Out o;
        o.put(kPod5Signature, 8);
        o.put(marker, 16);
        struct Entry {
            int64_t offset, length;
            int type;
        };
        std::vector<Entry> entries;
        {
            const std::vector<uint8_t> st = write_signal_table(signal_type, rows, read_ids, samples, offsets, data,
                                                               rows_per_batch, schema_md, footer_md, positions);
            if (positions)
                for (uint64_t i = 0; i < rows; i++) positions[i] += (uint64_t)o.b.size();
            if (!write) return (int)PGN_OK;
            entries.push_back({(int64_t)o.b.size(), (int64_t)st.size(), PGN_POD5_CONTENT_SIGNAL});
            o.put(st.data(), st.size());
            o.pad(8);
            o.put(marker, 16);
        }
        if (source)
            for (size_t i = 0; i < source->embedded.size(); i++) {
                if ((int)i == source->signal_index) continue;
                const auto& e = source->embedded[i];
                if (readsTable && e.content_type == PGN_POD5_CONTENT_READS) {  // a keep-going copy's reads
                    entries.push_back({(int64_t)o.b.size(), (int64_t)readsTable->size(), e.content_type});
                    o.put(readsTable->data(), readsTable->size());
                } else {
                    entries.push_back({(int64_t)o.b.size(), e.length, e.content_type});
                    o.put(source->raw.data() + e.offset, (size_t)e.length);
                }
                o.pad(8);
                o.put(marker, 16);
            }
        // footer (combined_file_utils.h:85-151)
        std::vector<FbNodeP> files;
        for (const Entry& e : entries) {
            auto t = fb_new_table();
            fb_add(t, 0, 8, (uint64_t)e.offset);
            fb_add(t, 1, 8, (uint64_t)e.length);
            fb_add(t, 2, 2, 0);  // FeatherV2
            fb_add(t, 3, 2, (uint64_t)(uint16_t)e.type);
            files.push_back(t);
        }
        auto ft = fb_new_table();
        fb_add(ft, 0, fb_new_string(ident));
        fb_add(ft, 1, fb_new_string(sw));
        fb_add(ft, 2, fb_new_string(ver));
        fb_add(ft, 3, fb_new_vec(files));
        const std::vector<uint8_t> fbf = FbBuilder::finish(ft);
        o.put("FOOTER\0\0", 8);
        o.put(fbf.data(), fbf.size());
        o.pad(8);
        const int64_t flen = (int64_t)fbf.size();
        o.put(&flen, 8);
        o.put(marker, 16);
        o.put(kPod5Signature, 8);
        FILE* fp = fopen(path, "wb");
        if (!fp) throw Pod5Error(PGN_ERR_IO, std::string("cannot create ") + path);
        const size_t w = fwrite(o.b.data(), 1, o.b.size(), fp);
        const int c = fclose(fp);
        if (w != o.b.size() || c != 0) throw Pod5Error(PGN_ERR_IO, std::string("cannot write ") + path);
        return (int)PGN_OK;
    });
}

int pgn_pod5_write_file(const char* path, const pgn_pod5_file* source, int signal_type, uint64_t rows,
                        const uint8_t* read_ids, const uint32_t* samples, const uint64_t* offsets, const uint8_t* data,
                        uint32_t rows_per_batch, const char* software, const uint8_t* section_marker)
{
    if (rows && offsets && offsets[rows] > offsets[0] && !data) return PGN_ERR_INVALID_ARG;
    return write_file_impl(path, source, signal_type, rows, read_ids, samples, offsets, data, rows_per_batch, software,
                           section_marker, true, nullptr);
}

int pgn_pod5_write_file_keep_going(const char* path, const pgn_pod5_file* source, int signal_type, uint64_t rows,
                                   const uint8_t* read_ids, const uint32_t* samples, const uint64_t* offsets,
                                   const uint8_t* data, const int32_t* row_status, uint32_t rows_per_batch,
                                   const uint8_t* section_marker, pgn_pod5_keep_going_result* res)
{
    if (!path || (rows && (!read_ids || !samples || !offsets || !row_status))) return PGN_ERR_INVALID_ARG;
    if (rows && offsets[rows] > offsets[0] && !data) return PGN_ERR_INVALID_ARG;  // as pgn_pod5_write_file
    return guarded([&] {
        pgn_pod5_keep_going_result r{0, 0, 0, 0, UINT64_MAX, 0, 0};
        std::vector<uint8_t> keepRow(rows, 0);
        std::vector<bool> keepRead;
        int iSignal = -1;
        std::unique_ptr<IpcReader> reads;
        if (source)
            for (const auto& e : source->embedded)
                if (e.content_type == PGN_POD5_CONTENT_READS) {
                    reads.reset(new IpcReader(source->raw.data() + e.offset, (size_t)e.length));
                    break;
                }
        if (reads) {
            for (size_t i = 0; i < reads->fields.size(); i++)
                if (reads->fields[i].name == "signal") iSignal = (int)i;
            if (iSignal < 0 || (reads->fields[iSignal].type != AT_List && reads->fields[iSignal].type != AT_LargeList) ||
                reads->fields[iSignal].dictionary || reads->fields[iSignal].children.size() != 1 ||
                reads->fields[iSignal].children[0].type != AT_Int || reads->fields[iSignal].children[0].int_bits != 64)
                corrupt("reads table: no signal list<uint64> column");
            // read batch by read batch, read by read: a read's rows are written until the first that
            // fails; then the read and the rest of its batch are not written (the reference's writer
            // stops pod5_add_reads_data there, c_api.cpp:1118-1127, and copy continues with the next
            // batch, copy.cpp:174-176).  The rows written before the failing one stay, listed by no read.
            std::vector<std::vector<int64_t>> lists;
            for (uint32_t b = 0; b < reads->batches.len; b++) {
                read_signal_lists(*reads, reads->block(reads->batches, b), iSignal, lists);
                bool failed = false;
                for (const auto& rl : lists) {
                    if (failed) {
                        keepRead.push_back(false);
                        r.dropped_reads++;
                        continue;
                    }
                    bool ok = true;
                    for (int64_t row : rl) {
                        if (row < 0 || (uint64_t)row >= rows) corrupt("reads table lists a signal row beyond the table");
                        if (row_status[row] != 0) {
                            if (r.first_failed_row == UINT64_MAX) {
                                r.first_failed_row = (uint64_t)row;
                                r.first_status = row_status[row];
                            }
                            ok = false;
                            break;
                        }
                        if (!keepRow[row]) keepRow[row] = 1;
                    }
                    if (!ok) {
                        // the rows kept so far for this read are orphans
                        for (int64_t row : rl) {
                            if (row_status[row] != 0) break;
                            r.orphan_rows++;
                        }
                        failed = true;
                        r.failed_batches++;
                        r.dropped_reads++;
                    }
                    keepRead.push_back(ok);
                }
            }
            // rows no read lists are written when they transcoded (as the plain transcode writes them)
            std::vector<uint8_t> listed(rows, 0);
            for (uint32_t b = 0; b < reads->batches.len; b++) {
                read_signal_lists(*reads, reads->block(reads->batches, b), iSignal, lists);
                for (const auto& rl : lists)
                    for (int64_t row : rl) listed[row] = 1;
            }
            for (uint64_t i = 0; i < rows; i++) {
                if (!listed[i] && row_status[i] == 0) keepRow[i] = 1;
                // a failing row no read lists is dropped too: reported like the listed ones
                if (!listed[i] && row_status[i] != 0 && r.first_failed_row == UINT64_MAX) {
                    r.first_failed_row = i;
                    r.first_status = row_status[i];
                }
            }
        } else {  // no reads table: every row stands alone
            for (uint64_t i = 0; i < rows; i++) {
                keepRow[i] = row_status[i] == 0;
                if (!keepRow[i] && r.first_failed_row == UINT64_MAX) {
                    r.first_failed_row = i;
                    r.first_status = row_status[i];
                }
            }
        }
        std::vector<int64_t> remap(rows, -1);
        uint64_t kept = 0;
        for (uint64_t i = 0; i < rows; i++)
            if (keepRow[i]) remap[i] = (int64_t)kept++;
        r.dropped_rows = rows - kept;
        if (res) *res = r;
        std::vector<uint8_t> nIds(16 * kept), nData;
        std::vector<uint32_t> nSamples(kept);
        std::vector<uint64_t> nOffs(kept + 1, 0);
        for (uint64_t i = 0, k = 0; i < rows; i++) {
            if (!keepRow[i]) continue;
            if (offsets[i + 1] < offsets[i]) return (int)PGN_ERR_INVALID_ARG;
            memcpy(nIds.data() + 16 * k, read_ids + 16 * i, 16);
            nSamples[k] = samples[i];
            nData.insert(nData.end(), data + offsets[i], data + offsets[i + 1]);
            nOffs[k + 1] = nData.size();
            k++;
        }
        std::vector<uint8_t> newReads;
        const bool rewrite = reads && kept != rows;
        if (rewrite) newReads = filter_reads_table(*reads, iSignal, keepRead, remap);
        return write_file_impl(path, source, signal_type, kept, nIds.data(), nSamples.data(), nOffs.data(),
                               nData.data(), rows_per_batch ? rows_per_batch : PGN_POD5_DEFAULT_SIGNAL_BATCH_ROWS,
                               nullptr, section_marker, true, nullptr, rewrite ? &newReads : nullptr);
    });
}

int pgn_pod5_write_file_reserved(const char* path, const pgn_pod5_file* source, int signal_type, uint64_t rows,
                                 const uint8_t* read_ids, const uint32_t* samples, const uint64_t* offsets,
                                 uint32_t rows_per_batch, const char* software, const uint8_t* section_marker,
                                 int write, uint64_t* row_positions)
{
    return write_file_impl(path, source, signal_type, rows, read_ids, samples, offsets, nullptr, rows_per_batch,
                           software, section_marker, write != 0, row_positions);
}

}  // extern "C"
