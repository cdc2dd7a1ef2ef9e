// ndfl_plugin.cpp -- the compressor plugin API of the reference on
// top of the GPU encoders: Strategy.decide(b, off, historyLen, dataLen) -> Decision, with
// Decision.getBitLengths() and Decision.compressTo(BitOutputStream, isFinal)
// (D/comp/Strategy.java:14, D/comp/Decision.java:16-19, D/comp/BitOutputStream.java:16-19).
//
// A strategy is a tree of ndfl_strategy_node: Lz77Huffman and Uncompressed leaves, MultiStrategy
// and BinarySplit inner nodes (include/ndfl.h).  decide() builds the reference's Decision tree:
// every Lz77Huffman leaf is encoded once on the GPU (ndfl_deflate_chunks_lz77, block at bit 0;
// its bits do not depend on the output position, only the bfinal bit on isFinal), Uncompressed
// leaves are closed forms, and the inner nodes combine their children's 8 bit lengths exactly as
// D/comp/MultiStrategy.java:31-57 and D/comp/BinarySplit.java:30-82 do (including BinarySplit's
// accumulation that indexes every child's lengths from position 0).  compressTo() walks the tree
// for the actual bit position and writes the chosen blocks through a host BitOut.
// This is the per-chunk, any-strategy path (user strategies mix in through the host mirror); the
// batched paths (ndfl_deflate_chunks*, ndfl_deflate_chunks_multi/_binsplit) stay the fast ones.
// D/ = /root/reference/src/io/nayuki/deflate/
#include <memory>
#include <vector>

struct ndfl_decision {
    uint64_t bits[8];
    int kind;                                   // NDFL_KIND_*
    // Lz77Huffman leaf: the block encoded at bit 0 as a non-final block
    std::vector<uint8_t> enc;
    uint64_t nbits = 0;
    // Uncompressed leaf: the data bytes (the caller's buffer, as the Java Decision closes over b)
    const uint8_t* data = nullptr;
    uint32_t len = 0;
    // MultiStrategy: the subdecision chosen per starting bit position
    std::shared_ptr<ndfl_decision> pick[8];
    // BinarySplit: per starting bit position, the block sequence (1: unsplit, 2: halves)
    std::vector<std::shared_ptr<ndfl_decision>> seq[8];
};

namespace plugin {

// BitOutputStream / DeflaterOutputStream.BitOut (D/DeflaterOutputStream.java:141-171): LSB-first.
struct BitOut {
    uint8_t* out;
    uint64_t cap;        // bytes
    uint64_t pos;        // bits written (incl. the start offset)
    bool overflow = false;
    void write(uint32_t v, uint32_t n) {          // 0 <= n <= 31
        uint32_t acc = n < 32 ? v & ((1u << n) - 1u) : v;
        while (n) {
            const uint64_t B = pos >> 3;
            const uint32_t sh = (uint32_t)(pos & 7), k = std::min(n, 8 - sh);
            if (B >= cap) { overflow = true; pos += n; return; }
            if (sh == 0) out[B] = 0;
            out[B] |= (uint8_t)((acc & ((1u << k) - 1u)) << sh);
            acc >>= k; n -= k; pos += k;
        }
    }
    // append `nbits` bits of `src` (bit 0 = src[0] bit 0); `first_or` is ORed into bit 0 (bfinal)
    void append(const uint8_t* src, uint64_t nbits, uint32_t first_or) {
        for (uint64_t k = 0; 8 * k < nbits; k++) {
            const uint32_t take = (uint32_t)std::min<uint64_t>(8, nbits - 8 * k);
            write((uint32_t)src[k] | (k == 0 ? first_or : 0u), take);
        }
    }
};

constexpr int MAX_BLOCK_LEN = 65535;            // Uncompressed.MAX_BLOCK_LEN (D/comp/Uncompressed.java:54)
constexpr int MAX_DEPTH = 64;

struct Ctx {
    ndfl_ctx* c;
    const ndfl_strategy_node* nodes;
    uint32_t n;
    int err = 0;
};

static int validate(const Ctx& X, uint32_t i, int depth) {
    if (i >= X.n || depth > MAX_DEPTH) return NDFL_E_ARG;
    const ndfl_strategy_node& s = X.nodes[i];
    switch (s.kind) {
        case NDFL_KIND_LZ77: {
            // Lz77Huffman's record validation (D/comp/Lz77Huffman.java:28-39): all zero (literal only)
            // or 3 <= minRun <= maxRun <= 258, 1 <= minDist <= maxDist <= 32768
            const bool lit = s.min_run == 0 && s.max_run == 0 && s.min_dist == 0 && s.max_dist == 0;
            if (!lit && !(3 <= s.min_run && s.min_run <= s.max_run && s.max_run <= 258 && 1 <= s.min_dist &&
                          s.min_dist <= s.max_dist && s.max_dist <= 32768))
                return NDFL_E_ARG;
            return 0;
        }
        case NDFL_KIND_UNCOMPRESSED: return 0;
        case NDFL_KIND_MULTI: {
            if (s.n_children < 1) return NDFL_E_ARG;            // "Empty list of strategies"
            for (int k = 0; k < s.n_children; k++) {
                const int e = validate(X, (uint32_t)(s.first_child + k), depth + 1);
                if (e) return e;
            }
            return 0;
        }
        case NDFL_KIND_BINSPLIT:
            if (s.min_block_len < 1) return NDFL_E_ARG;          // "Non-positive minimum block length"
            return validate(X, (uint32_t)s.first_child, depth + 1);
        default: return NDFL_E_ARG;
    }
}

using DecP = std::shared_ptr<ndfl_decision>;

static DecP decide(Ctx& X, uint32_t i, const uint8_t* b, uint64_t off, uint64_t hist, uint32_t len);

// Lz77Huffman.decide (D/comp/Lz77Huffman.java:42-59): the block encoded on the GPU.  The history
// the encoder may use is the last min(32768, historyLen) bytes (runs reach back one byte, matches at
// most 32768).
static DecP decide_lz(Ctx& X, const ndfl_strategy_node& s, const uint8_t* b, uint64_t off, uint64_t hist,
                      uint32_t len) {
    auto d = std::make_shared<ndfl_decision>();
    d->kind = NDFL_KIND_LZ77;
    const uint32_t hl = (uint32_t)std::min<uint64_t>(hist, 32768);
    const uint8_t* data = b + off + hist;
    const uint64_t cap = ndfl_deflate_bound(len, std::max<uint32_t>(len, 1)) + 16;
    d->enc.assign(cap, 0);
    uint64_t endb = 0;
    // an empty block can only be written as a final one by the batched encoder: clear bfinal after
    const int final_flag = len == 0 ? 1 : 0;
    const int r = ndfl_deflate_chunks_lz77(X.c, hl ? data - hl : nullptr, hl, hl ? 32768u : 0u, data, len,
                                           std::max<uint32_t>(len, 1), s.dynamic, s.min_run, s.max_run, s.min_dist,
                                           s.max_dist, final_flag, 0, d->enc.data(), cap, &endb, nullptr, 0);
    if (r) { X.err = r; return nullptr; }
    if (final_flag) d->enc[0] &= 0xFE;
    d->nbits = endb;
    d->enc.resize((endb + 7) / 8);
    for (int k = 0; k < 8; k++) d->bits[k] = endb;
    return d;
}

// Uncompressed.decide (D/comp/Uncompressed.java:22-51)
static DecP decide_unc(const uint8_t* b, uint64_t off, uint64_t hist, uint32_t len) {
    auto d = std::make_shared<ndfl_decision>();
    d->kind = NDFL_KIND_UNCOMPRESSED;
    d->data = b + off + hist;
    d->len = len;
    const int64_t numBlocks = std::max<int64_t>(((int64_t)len + MAX_BLOCK_LEN - 1) / MAX_BLOCK_LEN, 1);
    for (int i = 0; i < 8; i++) d->bits[i] = (uint64_t)((int64_t)len * 8 + numBlocks * 40 + ((13 - i) % 8 - 5));
    return d;
}

// MultiStrategy.decide (D/comp/MultiStrategy.java:31-57): per position the first substrategy with
// the fewest bits
static DecP decide_multi(Ctx& X, const ndfl_strategy_node& s, const uint8_t* b, uint64_t off, uint64_t hist,
                         uint32_t len) {
    auto d = std::make_shared<ndfl_decision>();
    d->kind = NDFL_KIND_MULTI;
    for (int i = 0; i < 8; i++) d->bits[i] = UINT64_MAX;      // Long.MAX_VALUE
    for (int k = 0; k < s.n_children; k++) {
        DecP sub = decide(X, (uint32_t)(s.first_child + k), b, off, hist, len);
        if (!sub) return nullptr;
        for (int i = 0; i < 8; i++)
            if (sub->bits[i] < d->bits[i]) { d->bits[i] = sub->bits[i]; d->pick[i] = sub; }
    }
    return d;
}

// BinarySplit.decide (D/comp/BinarySplit.java:36-82)
static uint64_t split_bits(const DecP* decs) {
    uint64_t bitLen = 0;                       // (sic) each child indexed from position 0 onwards
    for (int k = 0; k < 2; k++) bitLen += decs[k]->bits[bitLen % 8];
    return bitLen;
}
static DecP decide_split_with(Ctx& X, const ndfl_strategy_node& s, const uint8_t* b, uint64_t off, uint64_t hist,
                              uint32_t len, DecP cur) {
    auto d = std::make_shared<ndfl_decision>();
    d->kind = NDFL_KIND_BINSPLIT;
    for (int i = 0; i < 8; i++) { d->seq[i] = {cur}; d->bits[i] = cur->bits[i]; }
    const uint32_t firstHalfLen = (len + 1) / 2, secondHalfLen = len - firstHalfLen;
    if (std::min(firstHalfLen, secondHalfLen) > (uint32_t)s.min_block_len) {
        DecP split[2] = {decide(X, (uint32_t)s.first_child, b, off, hist, firstHalfLen),
                         decide(X, (uint32_t)s.first_child, b, off, hist + firstHalfLen, secondHalfLen)};
        if (!split[0] || !split[1]) return nullptr;
        bool improved = false;
        for (int i = 0; i < 8; i++) improved |= split_bits(split) < d->bits[i];
        if (improved) {
            split[0] = decide_split_with(X, s, b, off, hist, firstHalfLen, split[0]);
            split[1] = decide_split_with(X, s, b, off, hist + firstHalfLen, secondHalfLen, split[1]);
            if (!split[0] || !split[1]) return nullptr;
        }
        for (int i = 0; i < 8; i++) {
            const uint64_t bl = split_bits(split);
            if (bl < d->bits[i]) { d->bits[i] = bl; d->seq[i] = {split[0], split[1]}; }
        }
    }
    return d;
}

static DecP decide(Ctx& X, uint32_t i, const uint8_t* b, uint64_t off, uint64_t hist, uint32_t len) {
    const ndfl_strategy_node& s = X.nodes[i];
    switch (s.kind) {
        case NDFL_KIND_LZ77: return decide_lz(X, s, b, off, hist, len);
        case NDFL_KIND_UNCOMPRESSED: return decide_unc(b, off, hist, len);
        case NDFL_KIND_MULTI: return decide_multi(X, s, b, off, hist, len);
        default: {
            DecP cur = decide(X, (uint32_t)s.first_child, b, off, hist, len);
            if (!cur) return nullptr;
            return decide_split_with(X, s, b, off, hist, len, cur);
        }
    }
}

// Decision.compressTo (D/comp/Decision.java:19) for each kind
static void compress_to(const ndfl_decision* d, BitOut& w, bool isFinal) {
    switch (d->kind) {
        case NDFL_KIND_LZ77:
            w.append(d->enc.data(), d->nbits, isFinal ? 1u : 0u);
            return;
        case NDFL_KIND_UNCOMPRESSED: {          // D/comp/Uncompressed.java:33-47
            uint32_t index = 0;
            const uint32_t end = d->len;
            do {
                const uint32_t n = std::min<uint32_t>(end - index, MAX_BLOCK_LEN);
                w.write((isFinal && n == end - index) ? 1 : 0, 1);
                w.write(0, 2);
                w.write(0, (uint32_t)((8 - (w.pos & 7)) % 8));
                w.write(n ^ 0x0000u, 16);
                w.write(n ^ 0xFFFFu, 16);
                w.append(d->data + index, 8ull * n, 0);
                index += n;
            } while (index < end);
            return;
        }
        case NDFL_KIND_MULTI:
            compress_to(d->pick[w.pos & 7].get(), w, isFinal);
            return;
        default: {
            const auto& decs = d->seq[w.pos & 7];
            for (size_t k = 0; k < decs.size(); k++) compress_to(decs[k].get(), w, isFinal && k + 1 == decs.size());
            return;
        }
    }
}

}  // namespace plugin

int ndfl_decide(ndfl_ctx* c, const ndfl_strategy_node* nodes, uint32_t n_nodes, uint32_t root, const uint8_t* b,
                uint64_t off, uint32_t history_len, uint32_t data_len, uint64_t* bit_lengths, ndfl_decision** out) {
    if (!c || !nodes || !bit_lengths || !out || (!b && (history_len || data_len))) return NDFL_E_ARG;
    if (data_len > 65536) return NDFL_E_UNSUPPORTED;
    *out = nullptr;
    plugin::Ctx X{c, nodes, n_nodes};
    const int v = plugin::validate(X, root, 0);
    if (v) return v;
    plugin::DecP d;
    try {
        d = plugin::decide(X, root, b, off, history_len, data_len);
    } catch (const std::bad_alloc&) {
        return NDFL_E_INTERNAL;
    }
    if (!d) return X.err ? X.err : NDFL_E_INTERNAL;
    for (int i = 0; i < 8; i++) bit_lengths[i] = d->bits[i];
    *out = new ndfl_decision(*d);
    return NDFL_OK;
}

int ndfl_compress_to(ndfl_ctx* c, const ndfl_decision* dec, int is_final, uint32_t start_bitpos, uint8_t* out,
                     uint64_t out_cap, uint64_t* out_end_bits) {
    if (!c || !dec || !out || !out_end_bits || start_bitpos > 7) return NDFL_E_ARG;
    plugin::BitOut w{out, out_cap, start_bitpos};
    if (out_cap) out[0] &= (uint8_t)((1u << start_bitpos) - 1u);    // bits below start_bitpos are the caller's
    plugin::compress_to(dec, w, is_final != 0);
    *out_end_bits = w.pos;
    return w.overflow ? NDFL_E_CAPACITY : NDFL_OK;
}

int ndfl_decision_free(ndfl_decision* dec) {
    delete dec;
    return NDFL_OK;
}
