/*
 * ndfl.h -- C ABI of the MI355X-native DEFLATE codec (libndfl.so).
 *
 * This is the drop-in boundary for nayuki/DEFLATE-library-Java's encode/decode hot path.  Each
 * entry point names the reference interface it replaces (D/ = src/io/nayuki/deflate/ in the
 * reference).  Plain pointers and sizes only; no torch types.  Buffers are caller-owned; the
 * library never keeps a pointer past return.  A context owns device scratch and one HIP stream;
 * calls on one context are not reentrant, calls on different contexts are.
 *
 * Return convention (all int-returning calls):
 *     0                 success
 *     1 .. 19           DataFormatException.Reason ordinal + 1 (D/DataFormatException.java:61-83)
 *     < 0               NDFL_E_* (usage / device errors; map to IllegalArgument/IOException)
 */
#ifndef NDFL_H
#define NDFL_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define NDFL_ABI_VERSION 1u

/* error codes */
#define NDFL_OK               0
#define NDFL_E_ARG          (-1)   /* IllegalArgumentException / NullPointerException */
#define NDFL_E_UNSUPPORTED  (-2)   /* configuration not implemented on the GPU path */
#define NDFL_E_CAPACITY     (-3)   /* output buffer too small; required size reported */
#define NDFL_E_DEVICE       (-4)   /* HIP runtime error (IOException) */
#define NDFL_E_STATE        (-5)   /* IllegalStateException (use after finish/close) */
#define NDFL_E_INTERNAL     (-6)

/* DataFormatException.Reason ordinal + 1 */
enum ndfl_reason {
    NDFL_UNEXPECTED_END_OF_STREAM = 1, NDFL_RESERVED_BLOCK_TYPE, NDFL_UNCOMPRESSED_BLOCK_LENGTH_MISMATCH,
    NDFL_HUFFMAN_CODE_UNDER_FULL, NDFL_HUFFMAN_CODE_OVER_FULL, NDFL_NO_PREVIOUS_CODE_LENGTH_TO_COPY,
    NDFL_CODE_LENGTH_CODE_OVER_FULL, NDFL_END_OF_BLOCK_CODE_ZERO_LENGTH, NDFL_RESERVED_LENGTH_SYMBOL,
    NDFL_RESERVED_DISTANCE_SYMBOL, NDFL_LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE,
    NDFL_COPY_FROM_BEFORE_DICTIONARY_START, NDFL_HEADER_CHECKSUM_MISMATCH, NDFL_UNSUPPORTED_COMPRESSION_METHOD,
    NDFL_DECOMPRESSED_CHECKSUM_MISMATCH, NDFL_DECOMPRESSED_SIZE_MISMATCH, NDFL_GZIP_INVALID_MAGIC_NUMBER,
    NDFL_GZIP_RESERVED_FLAGS_SET, NDFL_GZIP_UNSUPPORTED_OPERATING_SYSTEM
};

/* Strategy ids: the Lz77Huffman presets (D/comp/Lz77Huffman.java:298-305) and Uncompressed. */
enum ndfl_strategy {
    NDFL_LITERAL_STATIC = 0, NDFL_LITERAL_DYNAMIC = 1, NDFL_RLE_STATIC = 2, NDFL_RLE_DYNAMIC = 3,
    NDFL_FULL_STATIC = 4, NDFL_FULL_DYNAMIC = 5, NDFL_UNCOMPRESSED = 6
};

/* memory flags */
#define NDFL_IN_DEVICE   1u    /* input pointers (data, hist) are device memory */
#define NDFL_OUT_DEVICE  2u    /* output pointer is device memory */
#define NDFL_DICT_DEFERRED 4u  /* ndfl_inflate_range: window bytes are written later (see resolve) */
#define NDFL_IN_PADDED   8u    /* ndfl_inflate / ndfl_inflate_range with NDFL_IN_DEVICE: the input is
                                 16-byte aligned and followed by NDFL_IN_PAD_BYTES readable zero bytes,
                                 so it is decoded in place (no staging copy); otherwise ignored */
#define NDFL_IN_PAD_BYTES 256u
#define NDFL_IN_PARTIAL  16u   /* ndfl_inflate_range: `in` is a prefix of the stream (more input may
                                 follow); see NDFL_NEED_INPUT */

/* ndfl_inflate_range with NDFL_IN_PARTIAL: the decode ran out of input inside a block.  Nothing is
 * reported for that block: *consumed_bits is its start (the last block boundary reached) and
 * *out_len the bytes decoded before it.  The caller continues from there with more input and the
 * last <= 32 KiB of output as the window -- Open.read's incremental refill
 * (D/decomp/Open.java:137-192) at block granularity.  Not a Reason: at true end of input the
 * caller decodes without the flag and gets UNEXPECTED_END_OF_STREAM. */
#define NDFL_NEED_INPUT  64

typedef struct ndfl_ctx ndfl_ctx;

uint32_t ndfl_abi_version(void);
const char* ndfl_error_string(int code);

/* Create a context on HIP device `device`.  Fails with NDFL_E_DEVICE if no GPU.
 * The NDFL_* environment switches (test hand-over paths, statistics, A/B alternatives: the Knobs of
 * csrc/hip/ndfl_common.hpp; none is needed in production) are read ONCE, here: setting or changing
 * one after a context exists has no effect on it -- create a new context to measure another
 * setting.  A switch is on when set to anything but "0".  With NDFL_STATS on, the context prints its
 * effective switches once to stderr, so a profiling run shows which path it measured. */
int ndfl_ctx_create(ndfl_ctx** out, int device, uint32_t flags);
int ndfl_ctx_destroy(ndfl_ctx* ctx);
/*
 * Stream ordering (every call that reads or writes device memory: NDFL_IN_DEVICE / NDFL_OUT_DEVICE
 * buffers, ndfl_bits_shift, the deferred-window resolve).  By default a call's device work is
 * ordered after all work queued earlier on the device's default (NULL) stream, so a buffer just
 * produced there -- or a freed block a caching allocator hands out again while a kernel on that
 * stream still uses it -- is safe to pass without a host synchronize.  A caller that works on
 * another stream names it with ndfl_ctx_set_stream: the calls then run on that stream, in order
 * with the caller's own work (NULL restores the default).  Every call completes its device work
 * before it returns, so its outputs may be used right away on any stream.
 */
int ndfl_ctx_set_stream(ndfl_ctx* ctx, void* hip_stream);
/* Average device time (ms) of the last call's dominant kernel, measured with HIP events. */
double ndfl_ctx_last_kernel_ms(ndfl_ctx* ctx);
/* Device-time breakdown of the last calls (ms): [0] deflate kernel, [1] inflate finder,
 * [2] inflate count, [3] inflate emit, [4] inflate device span, [5] linked chains, [6] repaired
 * boundaries, [7] header candidates, [8] chains whose first block the count pass decoded one lane
 * per block (escape-prefix literal codes).  Returns the number of entries written (<= 9). */
int ndfl_ctx_timings(ndfl_ctx* ctx, double* ms, int n);
/* The reserved symbol behind the last ndfl_inflate / ndfl_inflate_range that returned
 * NDFL_RESERVED_LENGTH_SYMBOL (286 or 287) or NDFL_RESERVED_DISTANCE_SYMBOL (30 or 31), else -1:
 * the reference's message names it -- "Reserved run length symbol: " + sym,
 * "Reserved distance symbol: " + sym (D/decomp/Open.java:516, 550, 659, 674). */
int ndfl_ctx_error_symbol(ndfl_ctx* ctx);

/*
 * Compress K consecutive chunks of one DEFLATE stream.
 * Replaces K iterations of DeflaterOutputStream.writeBuffer (D/DeflaterOutputStream.java:119-137),
 * i.e. Strategy.decide(b, off, historyLen, dataLen) + Decision.compressTo(bitOut, isFinal)
 * (D/comp/Strategy.java:14, D/comp/Decision.java:16-19, D/comp/Lz77Huffman.java:42-286) and the
 * BitOut packing (D/DeflaterOutputStream.java:141-171).  Batching is exact because the default
 * decisions depend only on raw input, never on earlier output.
 *   hist/hist_len   the min(historyLookbehindLimit, pos) raw bytes preceding `data`
 *   data/len        K chunks: chunk_len bytes each, the last one 0..chunk_len bytes
 *   final_flag      1 if the last chunk is the stream's final chunk (bfinal=1); if 0, every
 *                   chunk must be full (len % chunk_len == 0, len > 0)
 *   hist_limit      historyLookbehindLimit (0..32768) -- decides whether history exists
 *   start_bitpos    BitOutputStream.getBitPosition() before the first block (0..7): the output
 *                   begins at that bit of out[0]; bits below it are written as 0 (caller ORs)
 *   out/out_cap     output bytes; on success *out_end_bits = start_bitpos + bits written
 *   crc_inout       optional: java.util.zip.CRC32 value updated with `data` (GzipOutputStream)
 * Returns 0, NDFL_E_UNSUPPORTED (chunk_len > 65536), NDFL_E_CAPACITY
 * (*out_end_bits = bits required), ...  FULL_STATIC / FULL_DYNAMIC run ndfl_deflate_chunks_lz77
 * with (3, 258, 1, 32768).
 */
int ndfl_deflate_chunks(ndfl_ctx* ctx, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                        const uint8_t* data, uint64_t len, uint32_t chunk_len, int strategy,
                        int final_flag, uint32_t start_bitpos, uint8_t* out, uint64_t out_cap,
                        uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags);

/*
 * Same as ndfl_deflate_chunks for an explicit Lz77Huffman(useDynamicHuffmanCodes,
 * searchMinimumRunLength, searchMaximumRunLength, searchMinimumDistance, searchMaximumDistance)
 * strategy (D/comp/Lz77Huffman.java:20-39 record + validation, :62-130 greedy longest-match parse
 * with the smallest distance on ties).  (0,0,0,0) is the literal-only form; parameters outside
 * 3 <= minRun <= maxRun <= 258, 1 <= minDist <= maxDist <= 32768 give NDFL_E_ARG
 * (IllegalArgumentException, :37-38).  The FULL_* presets are (3, 258, 1, 32768).
 */
int ndfl_deflate_chunks_lz77(ndfl_ctx* ctx, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                             const uint8_t* data, uint64_t len, uint32_t chunk_len, int dynamic, int min_run,
                             int max_run, int min_dist, int max_dist, int final_flag, uint32_t start_bitpos,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_end_bits, uint32_t* crc_inout,
                             uint32_t flags);

/* A substrategy of ndfl_deflate_chunks_multi: an Lz77Huffman record or Uncompressed.SINGLETON. */
#define NDFL_KIND_LZ77          0
#define NDFL_KIND_UNCOMPRESSED  1
typedef struct {
    int32_t kind;                                     /* NDFL_KIND_* */
    int32_t dynamic, min_run, max_run, min_dist, max_dist;   /* Lz77Huffman components (kind LZ77) */
} ndfl_strategy_desc;

/*
 * Same as ndfl_deflate_chunks for a MultiStrategy(strats...) (D/comp/MultiStrategy.java:31-57)
 * over up to 8 Lz77Huffman / Uncompressed substrategies (n_strats = 1 gives that strategy alone):
 * per chunk, the first substrategy with the fewest bits at the current output bit position
 * (Decision.getBitLengths, D/comp/Decision.java:16-19; Uncompressed's depend on the position,
 * D/comp/Uncompressed.java:22-26).  NDFL_UNCOMPRESSED in ndfl_deflate_chunks runs this with the
 * single Uncompressed substrategy.
 */
int ndfl_deflate_chunks_multi(ndfl_ctx* ctx, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                              const uint8_t* data, uint64_t len, uint32_t chunk_len, const ndfl_strategy_desc* strats,
                              uint32_t n_strats, int final_flag, uint32_t start_bitpos, uint8_t* out,
                              uint64_t out_cap, uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags);

/*
 * Same as ndfl_deflate_chunks for BinarySplit(sub, minBlockLen) (D/comp/BinarySplit.java:21-82) over
 * an Lz77Huffman substrategy: each chunk halves recursively while both halves exceed
 * min_block_len (>= 1, else NDFL_E_ARG), keeping a split when it takes fewer bits; the sub-blocks'
 * history starts at their chunk's.  NDFL_E_UNSUPPORTED for other substrategies, for halvings of
 * an odd length inside full chunks, or for more than 8192 node encodes in a partial final chunk.
 */
int ndfl_deflate_chunks_binsplit(ndfl_ctx* ctx, const uint8_t* hist, uint32_t hist_len, uint32_t hist_limit,
                                 const uint8_t* data, uint64_t len, uint32_t chunk_len, const ndfl_strategy_desc* sub,
                                 int32_t min_block_len, int final_flag, uint32_t start_bitpos, uint8_t* out,
                                 uint64_t out_cap, uint64_t* out_end_bits, uint32_t* crc_inout, uint32_t flags);

/*
 * The compressor plugin API (D/comp/Strategy.java:14, D/comp/Decision.java:16-19): one chunk,
 * any strategy tree.  A strategy is an array of nodes; node `root` is the strategy:
 *   NDFL_KIND_LZ77          Lz77Huffman(dynamic, min_run, max_run, min_dist, max_dist)
 *   NDFL_KIND_UNCOMPRESSED  Uncompressed.SINGLETON
 *   NDFL_KIND_MULTI         MultiStrategy(nodes[first_child .. first_child + n_children))
 *   NDFL_KIND_BINSPLIT      BinarySplit(nodes[first_child], min_block_len)
 * ndfl_decide = Strategy.decide(b, off, historyLen, dataLen) on the GPU encoders: the data is
 * b[off + history_len, + data_len) (host memory, <= 65536 bytes), preceded by its history;
 * bit_lengths[i] = Decision.getBitLengths()[i], the block's bits when it starts at bit position
 * i (mod 8).  The decision keeps a pointer to `b` (as the Java Decision closes over it): keep b
 * valid until the decision is freed.  NDFL_E_ARG for the constructors' IllegalArgumentExceptions
 * (Lz77Huffman parameters, empty MultiStrategy, minBlockLen < 1) and malformed trees.
 * ndfl_compress_to = Decision.compressTo(out, isFinal): writes the block(s) at bit start_bitpos of
 * out[0] (lower bits kept), *out_end_bits = start_bitpos + bits written.
 */
#define NDFL_KIND_MULTI         2
#define NDFL_KIND_BINSPLIT      3
typedef struct {
    int32_t kind;                                        /* NDFL_KIND_* */
    int32_t dynamic, min_run, max_run, min_dist, max_dist;   /* LZ77 */
    int32_t first_child, n_children;                     /* MULTI / BINSPLIT (n_children unused) */
    int32_t min_block_len;                               /* BINSPLIT */
} ndfl_strategy_node;
typedef struct ndfl_decision ndfl_decision;
int ndfl_decide(ndfl_ctx* ctx, const ndfl_strategy_node* nodes, uint32_t n_nodes, uint32_t root, const uint8_t* b,
                uint64_t off, uint32_t history_len, uint32_t data_len, uint64_t* bit_lengths, ndfl_decision** out);
int ndfl_compress_to(ndfl_ctx* ctx, const ndfl_decision* dec, int is_final, uint32_t start_bitpos, uint8_t* out,
                     uint64_t out_cap, uint64_t* out_end_bits);
int ndfl_decision_free(ndfl_decision* dec);

/* Upper bound of output bytes of ndfl_deflate_chunks for `len` bytes. */
uint64_t ndfl_deflate_bound(uint64_t len, uint32_t chunk_len);

/*
 * Decompress one raw DEFLATE stream held entirely in `in`.
 * Replaces InflaterInputStream.read / Open.read (D/InflaterInputStream.java:147-164,
 * D/decomp/Open.java:83-124) run to end of stream.  Trailing bytes after the final block are
 * ignored; *consumed_bits is the bit position just after the final block (endExactly
 * repositioning uses ceil(consumed_bits/8), D/decomp/Open.java:113-124).
 * Returns 0, a Reason code (with *out_len = bytes decoded before the error), NDFL_E_CAPACITY
 * (*out_len = bytes required), or a negative error.
 */
int ndfl_inflate(ndfl_ctx* ctx, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
                 uint64_t* out_len, uint64_t* consumed_bits, uint32_t flags);

/*
 * Decompress the block-aligned bit range [start_bit, end_bit) of one raw DEFLATE stream: one GPU's
 * shard of a stream decoded across GPUs, or one batch of a stream read incrementally
 * (NDFL_IN_PARTIAL, end_bit UINT64_MAX: InflaterInputStream's bounded input buffer,
 * D/InflaterInputStream.java:96-106).  For the multi-GPU case: one GPU's
 * shard of a stream decoded across GPUs.  Same decoder as ndfl_inflate, i.e.
 * Open.read (D/decomp/Open.java:83-124), started at a block boundary with the reference's
 * dictionary state (the 32 KiB ring, :592-603) given by the caller instead of built up.
 *   out         window start: out[0, dict_len) holds the dict_len (<= 32768) output bytes preceding
 *               the range; decoded bytes are written to out[dict_len, dict_len + *out_len)
 *   end_bit     stop at the block boundary == end_bit (UINT64_MAX: run to the final block);
 *               NDFL_E_ARG if a block straddles it
 *   flags       NDFL_DICT_DEFERRED (requires NDFL_OUT_DEVICE): the window is not written yet.  The
 *               call decodes everything, records which chains of blocks read the window (directly
 *               or through other chains), and ndfl_inflate_resolve re-emits exactly those after the
 *               caller has written it; so all GPUs decode in parallel and only the window (32 KiB)
 *               is passed along.  `in` and `out` must stay valid until the resolve call.
 * Returns as ndfl_inflate (COPY_FROM_BEFORE_DICTIONARY_START counts the window as dictionary).
 */
int ndfl_inflate_range(ndfl_ctx* ctx, const uint8_t* in, uint64_t in_len, uint64_t start_bit, uint64_t end_bit,
                       uint8_t* out, uint64_t dict_len, uint64_t out_cap, uint64_t* out_len,
                       uint64_t* consumed_bits, uint32_t flags);
/*
 * Multi-GPU decode of a stream WITHOUT a seam index (SURVEY §8e decompress): a block boundary
 * at or past from_bit that the decoder has confirmed -- the end of a chain of blocks, decoded from
 * a header candidate (the reference's own header checks, D/decomp/Open.java:322-435), that lands
 * exactly on another candidate whose own chain links on (or is final) -- looking at most
 * window_bits ahead;
 * *sync_bit = UINT64_MAX if there is none.  GPU r of N takes [sync(r*C/N), sync((r+1)*C/N)) and
 * decodes it with ndfl_inflate_range (deferred window); ndfl_inflate_range's exact-boundary
 * check (NDFL_E_ARG when a block straddles end_bit) proves each seam, starting from bit 0.
 * flags: NDFL_IN_DEVICE / NDFL_IN_PADDED as for ndfl_inflate.
 */
int ndfl_inflate_sync(ndfl_ctx* ctx, const uint8_t* in, uint64_t in_len, uint64_t from_bit, uint64_t window_bits,
                      uint64_t* sync_bit, uint32_t flags);
/*
 * Diagnostics (no reference counterpart; used by the parity tests): the decoder's chain starts in
 * the raw DEFLATE stream `in` -- the bit positions at which the header finder and the strict stage
 * accept a block header, by the reference's own header checks (UncompressedBlock ctor
 * D/decomp/Open.java:232-241, HuffmanBlock(true) :336-431) restricted to headers a chain may start
 * at (BFINAL = 0; stored with zero padding, its LEN bytes in the input and a plausible next
 * header; dynamic with HLIT, HDIST < 30).  headers[0, min(cap, *n_headers)) = the positions in
 * ascending order, at most 256 per 64 KiB of input (the decoder's per-segment cap); survivors
 * (optional) = the finder's survivors before the strict stage (bit 63 set: dynamic); stats
 * (optional, 4 entries) = survivors found, headers accepted before the cap, segments over the cap,
 * survivors dropped past the survivor list's capacity.  flags: NDFL_IN_DEVICE / NDFL_IN_PADDED.
 */
int ndfl_inflate_headers(ndfl_ctx* ctx, const uint8_t* in, uint64_t in_len, uint32_t flags, uint64_t* headers,
                         uint64_t cap, uint64_t* n_headers, uint64_t* survivors, uint64_t surv_cap, uint64_t* stats);
/* Finish the last NDFL_DICT_DEFERRED range decode on this context (NDFL_E_STATE if none). */
int ndfl_inflate_resolve(ndfl_ctx* ctx, uint64_t* n_reemitted);
/*
 * Multi-GPU window chain: once the caller has written the window of the last
 * NDFL_DICT_DEFERRED range decode, dst[0, tail_len) (device memory) = the final values of the last
 * tail_len bytes of out[0, dict_len + out_len), without resolving the rest -- the next GPU's window,
 * passed on before this GPU's own resolve (ndfl_inflate_resolve still finishes the decode).  In the
 * reference this is the 32 KiB dictionary that Open carries from one block to the next
 * (D/decomp/Open.java:592-603).  NDFL_E_STATE if no deferred decode is pending, NDFL_E_UNSUPPORTED if
 * a byte's back-reference chain is too long to follow (resolve first, then take the bytes from out).
 */
int ndfl_inflate_tail(ndfl_ctx* ctx, uint64_t tail_len, uint8_t* dst);
/*
 * The window chain in one step: the same last tail_len bytes of the pending
 * NDFL_DICT_DEFERRED decode as a map of its window, before the window is written: dst[k] (device
 * memory, u32) = the window byte index (< dict_len) byte k's value comes from, or
 * NDFL_TAIL_LITERAL | value for a byte that does not depend on the window.  Every GPU computes its
 * map at once; an all-gather of the maps lets GPU r compose those of GPUs 0..r-1 into its window
 * (Open's 32 KiB dictionary, D/decomp/Open.java:592-603, carried across all earlier shards)
 * without waiting for GPU r-1.  Errors as ndfl_inflate_tail.
 */
#define NDFL_TAIL_LITERAL 0x80000000u
int ndfl_inflate_tail_map(ndfl_ctx* ctx, uint64_t tail_len, uint32_t* dst);

/*
 * Multi-GPU seam step for compression: place the first `nbits` bits of `in` at bit
 * `shift` (0..7) of out[0] (lower bits 0, bits past the end 0).  A shard compressed at bit 0 by
 * ndfl_deflate_chunks is thereby moved to its global bit offset mod 8; the byte shared with the
 * previous shard is ORed when the stream is assembled -- BitOut's byte packing
 * (D/DeflaterOutputStream.java:147-156) across GPUs.  Device pointers only (NDFL_IN_DEVICE |
 * NDFL_OUT_DEVICE), not in place.
 */
int ndfl_bits_shift(ndfl_ctx* ctx, const uint8_t* in, uint64_t nbits, uint32_t shift, uint8_t* out,
                    uint64_t out_cap, uint32_t flags);

/* java.util.zip.CRC32.update over a buffer, on the GPU (flags: NDFL_IN_DEVICE). */
int ndfl_crc32(ndfl_ctx* ctx, uint32_t* crc_inout, const uint8_t* data, uint64_t len, uint32_t flags);
/* java.util.zip.Adler32.update over a buffer, on the GPU (flags: NDFL_IN_DEVICE): the zlib
 * container's checksum (D/ZlibOutputStream.java:22,48, D/ZlibInputStream.java:25,57-69).
 * *adler_inout = (b << 16) | a, 1 for a fresh checksum. */
int ndfl_adler32(ndfl_ctx* ctx, uint32_t* adler_inout, const uint8_t* data, uint64_t len, uint32_t flags);
/* crc of A||B from crc(A), crc(B), |B| (host arithmetic). */
uint32_t ndfl_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

#ifdef __cplusplus
}
#endif
#endif
