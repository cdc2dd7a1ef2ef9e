/*
 * ndfl_oracle.h -- CPU restatement of nayuki/DEFLATE-library-Java's encode/decode path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the MI355X codec.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * library (deflate-library-java_amd/) never links or calls it.
 *
 * The reference is Java (JDK >= 18) and no JDK exists in this image, so it cannot be built or
 * run here (see DESIGN.md "Oracle").  Parity of this restatement is pinned by:
 *   - the 39 decoder known-answer tests of T/InflaterInputStreamTest.java (tests/golden/inflate_kat.json),
 *   - seeded restatements of that file's three random generators,
 *   - Python zlib 1.2.11 as an independent DEFLATE decoder/encoder for valid streams,
 *   - an independent pure-Python restatement of Lz77Huffman (N-version, byte-equal),
 *   - the hand-derived encoder known-answer tests of SURVEY.md App. A.8.
 *
 * Citations: D/ = /root/reference/src/io/nayuki/deflate/
 */
#ifndef NDFL_ORACLE_H
#define NDFL_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Strategy ids (D/comp/Lz77Huffman.java:298-305 presets, D/comp/Uncompressed.java). */
enum {
    OR_LITERAL_STATIC = 0, OR_LITERAL_DYNAMIC = 1,
    OR_RLE_STATIC = 2, OR_RLE_DYNAMIC = 3,
    OR_FULL_STATIC = 4, OR_FULL_DYNAMIC = 5,
    OR_UNCOMPRESSED = 6
};

/* Error codes: 1 + DataFormatException.Reason ordinal (D/DataFormatException.java:61-83). */
enum {
    OR_OK = 0,
    OR_UNEXPECTED_END_OF_STREAM = 1, OR_RESERVED_BLOCK_TYPE, OR_UNCOMPRESSED_BLOCK_LENGTH_MISMATCH,
    OR_HUFFMAN_CODE_UNDER_FULL, OR_HUFFMAN_CODE_OVER_FULL, OR_NO_PREVIOUS_CODE_LENGTH_TO_COPY,
    OR_CODE_LENGTH_CODE_OVER_FULL, OR_END_OF_BLOCK_CODE_ZERO_LENGTH, OR_RESERVED_LENGTH_SYMBOL,
    OR_RESERVED_DISTANCE_SYMBOL, OR_LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE,
    OR_COPY_FROM_BEFORE_DICTIONARY_START, OR_HEADER_CHECKSUM_MISMATCH, OR_UNSUPPORTED_COMPRESSION_METHOD,
    OR_DECOMPRESSED_CHECKSUM_MISMATCH, OR_DECOMPRESSED_SIZE_MISMATCH, OR_GZIP_INVALID_MAGIC_NUMBER,
    OR_GZIP_RESERVED_FLAGS_SET, OR_GZIP_UNSUPPORTED_OPERATING_SYSTEM
};
#define OR_ERR_CAPACITY (-1)
#define OR_ERR_ARG      (-2)

/* DeflaterOutputStream(out, chunkLen, histLimit, strategy) fed `len` bytes then finish()
 * (D/DeflaterOutputStream.java:55-171).  `brute` = 1 uses the reference's literal exhaustive
 * distance loop for FULL_* (D/comp/Lz77Huffman.java:71-84); 0 uses an exact-prefix chain walk
 * that visits every candidate (equivalent; pinned by tests).  Returns bytes written or <0. */
int64_t or_deflate(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                   int strategy, int brute, uint8_t* out, uint64_t out_cap);

/* Same as or_deflate but with explicit Lz77Huffman(dynamic,minRun,maxRun,minDist,maxDist). */
int64_t or_deflate_lz(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                      int dynamic, int min_run, int max_run, int min_dist, int max_dist, int brute,
                      uint8_t* out, uint64_t out_cap);

/* MultiStrategy(subs...) (D/comp/MultiStrategy.java:31-57) driven like DeflaterOutputStream; desc is
 * n x {kind (0 Lz77Huffman, 1 Uncompressed), dynamic, minRun, maxRun, minDist, maxDist}. */
int64_t or_deflate_multi(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                         const int32_t* desc, uint32_t n, uint8_t* out, uint64_t out_cap);

/* BinarySplit(sub, minBlockLen) (D/comp/BinarySplit.java:21-82) driven like DeflaterOutputStream;
 * desc = {kind (0 Lz77Huffman, 1 Uncompressed), dynamic, minRun, maxRun, minDist, maxDist}. */
int64_t or_deflate_binsplit(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                            const int32_t* desc, int32_t min_block_len, uint8_t* out, uint64_t out_cap);

/* Per-chunk bit sizes of the default encode (for GPU parity of block boundaries).  Writes
 * number of chunks to *nchunks and each chunk's block bit length into bits[] (cap entries). */
int64_t or_deflate_block_bits(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                              int strategy, uint64_t* bits, uint64_t cap);

/* Fixture generator: chunk i uses strategy strat[i % nstrat]. */
int64_t or_deflate_mixed(const uint8_t* data, uint64_t len, uint32_t chunk_len, uint32_t hist_limit,
                         const int8_t* strat, uint32_t nstrat, uint8_t* out, uint64_t out_cap);

/* InflaterInputStream over the whole of `in` (D/decomp/Open.java).  Returns 0 or 1+Reason.
 * *out_len = bytes produced before success/error; *consumed_bits = bit position after the
 * final block (meaningful on success).  OR_ERR_CAPACITY if out_cap is too small. */
int or_inflate(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
               uint64_t* out_len, uint64_t* consumed_bits);
/* Range form: start at start_bit with dict_len bytes of preceding output, stop at the block
 * boundary == end_bit (UINT64_MAX: after the final block). */
int or_inflate_range(const uint8_t* in, uint64_t in_len, uint64_t start_bit, uint64_t end_bit,
                     const uint8_t* dict, uint64_t dict_len, uint8_t* out, uint64_t out_cap,
                     uint64_t* out_len, uint64_t* consumed_bits);

/* Decoder test support (not a reference interface): every bit position p in [lo, hi) at which the
 * GPU decoder may start a chain of blocks, i.e. a block header the reference's checks accept
 * (UncompressedBlock ctor D/decomp/Open.java:232-241, HuffmanBlock(true) :336-431) that also passes
 * the decoder's chain-start filter: BFINAL = 0; stored: zero padding
 * bits, the LEN bytes inside the input, and a plausible next header (BTYPE != 3; stored: LEN ==
 * ~NLEN; dynamic: a complete code-length code); dynamic: HLIT < 30 and HDIST < 30.  Positions in
 * ascending order; returns their number (positions past `cap` are counted, not written). */
int64_t or_scan_headers(const uint8_t* in, uint64_t in_len, uint64_t lo, uint64_t hi, uint64_t* out, uint64_t cap);

/* K iterations of DeflaterOutputStream.writeBuffer (D/DeflaterOutputStream.java:119-137) on
 * `data` with the raw bytes `hist` before it (only its last min(hist_limit, .) bytes are used),
 * starting at bit 0: the semantics of ndfl_deflate_chunks.  final_flag = 0 requires whole chunks.
 * Writes ceil(bits/8) bytes (last byte zero-padded, no finish()); *out_bits = bits. */
int64_t or_deflate_chunks(const uint8_t* hist, uint64_t hist_len, const uint8_t* data, uint64_t len,
                          uint32_t chunk_len, uint32_t hist_limit, int strategy, int final_flag,
                          uint8_t* out, uint64_t out_cap, uint64_t* out_bits);

/* Checksums (JDK java.util.zip.CRC32 / Adler32 semantics: CRC-32/ISO-HDLC, Adler-32). */
uint32_t or_crc32(uint32_t crc, const uint8_t* p, uint64_t n);
uint32_t or_adler32(uint32_t adler, const uint8_t* p, uint64_t n);

/* GzipMetadata (D/GzipMetadata.java:30-39).  mtime 0 = absent; os: 0..13 or 255. */
typedef struct {
    int32_t is_text;
    int32_t has_mtime;  uint32_t mtime;
    int32_t extra_flags;
    int32_t os;
    int32_t has_extra; uint32_t extra_len; const uint8_t* extra;
    int32_t has_name;  const char* name;      /* ISO-8859-1 bytes, NUL-terminated */
    int32_t has_comment; const char* comment;
    int32_t has_header_crc;
} or_gzip_meta;

/* GzipOutputStream(new DeflaterOutputStream(out), meta) + write(all) + close
 * (D/GzipOutputStream.java:32-78, D/GzipMetadata.java:164-212). */
int64_t or_gzip_compress(const uint8_t* data, uint64_t len, const or_gzip_meta* meta,
                         uint8_t* out, uint64_t out_cap);

/* GzipInputStream read to EOF (D/GzipInputStream.java:38-90, D/GzipMetadata.java:73-146).
 * Returns 0 or 1+Reason; header fields are reported through hdr (string pointers point into
 * `in`).  *member_end = byte offset just after the trailer on success. */
int or_gunzip(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
              or_gzip_meta* hdr, uint64_t* member_end);

/* Zlib container (D/ZlibOutputStream.java, D/ZlibInputStream.java, D/ZlibMetadata.java). */
int64_t or_zlib_compress(const uint8_t* data, uint64_t len, int cinfo, int level,
                         uint8_t* out, uint64_t out_cap);
int or_zlib_decompress(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_cap,
                       uint64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif
