/* ctok.h -- C ABI of the MI355X-native batch ByteLevel-BPE encode path.
 *
 * Drop-in boundary for the reference's PyO3 class `complexity_tokenizer.Tokenizer`
 * (Complexity-ML/complexity-tokenizer v0.3.3, src/bindings/tokenizer.rs:11-14, registered at
 * src/lib.rs:49).  Every entry point below names the reference method it replaces.  Plain
 * pointers and sizes only; no torch or HIP types appear in the signatures (the stream is an
 * opaque `void*` that the library casts to hipStream_t).
 *
 * Ownership: a `ctok*` is immutable after creation and safe to share between threads; calls on
 * the same device serialise on that device's workspace.  Errors: every `int` return is 0
 * (CTOK_OK) or a negative CTOK_E_* code; ctok_last_error() returns the message of the calling
 * thread's last failure.
 */
#ifndef CTOK_H
#define CTOK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ctok ctok;

enum {
  CTOK_OK = 0,
  CTOK_E_IO = -1,          /* file open/read failure              -> Python IOError   */
  CTOK_E_PARSE = -2,       /* JSON / schema failure (serde error) -> Python IOError   */
  CTOK_E_UNSUPPORTED = -3, /* component outside the encode hot path (e.g. Metaspace)  */
  CTOK_E_ARG = -4,         /* bad argument (null pointer, unsorted offsets, ...)      */
  CTOK_E_CAPACITY = -5,    /* ids_cap too small; tok_off[n_docs] holds the size needed */
  CTOK_E_PANIC = -6,       /* the reference would panic (src/bpe.rs:141 index OOB)   */
  CTOK_E_DEVICE = -7,      /* HIP runtime failure                                     */
  CTOK_E_NOTFOUND = -8     /* token_to_id / id_to_token miss (Python None)            */
};

/* Message of the calling thread's last failing call ("" if none). */
const char* ctok_last_error(void);
/* Library version string, e.g. "0.3.3+mi355x.1". */
const char* ctok_version(void);

/* Tokenizer.from_file(path)                 src/bindings/tokenizer.rs:18-23
 *   -> HuggingFaceTokenizer::from_file       src/huggingface/mod.rs:159-166, :247-334 */
int ctok_create_from_file(const char* path, ctok** out);
/* HuggingFaceTokenizer::from_str / from_buffer   src/huggingface/mod.rs:168-180 */
int ctok_create_from_buffer(const char* json, size_t len, ctok** out);

/* A tokenizer from in-memory tables instead of tokenizer.json text: the same
 * loader (BpeTokenizer::new src/bpe.rs:52-79 with its rank quirks, added-token rules
 * src/huggingface/mod.rs:247-334) on the model a ByteLevel BPE tokenizer.json describes.
 *   vocab:  token i = vocab[vocab_off[i] .. vocab_off[i+1]) (its byte-level string), id vocab_id[i]
 *   merges: merge r joins the tokens with ids merge_left[r], merge_right[r] (rank order; the new
 *           token is the vocab entry of their concatenated strings, as for "a b" merge strings);
 *           CTOK_E_ARG when either token's string contains ' ' (the reference splits "a b" on ' '
 *           and silently drops such a merge, src/huggingface/mod.rs:252-264)
 *   added:  content i = added[added_off[i] .. added_off[i+1]), id added_id[i], CTOK_ADDED_* flags
 *   nfc:    1 = normalizer NFC, 0 = none; add_prefix_space: ByteLevel's flag */
enum {
  CTOK_ADDED_SPECIAL = 1,
  CTOK_ADDED_SINGLE_WORD = 2,
  CTOK_ADDED_LSTRIP = 4,
  CTOK_ADDED_RSTRIP = 8,
  CTOK_ADDED_NORMALIZED = 16
};
typedef struct ctok_tables {
  const char* vocab;
  const uint64_t* vocab_off;
  const uint32_t* vocab_id;
  uint64_t n_vocab;
  const uint32_t* merge_left;
  const uint32_t* merge_right;
  uint64_t n_merges;
  const char* added;
  const uint64_t* added_off;
  const uint32_t* added_id;
  const uint8_t* added_flags;
  uint64_t n_added;
  int nfc;
  int add_prefix_space;
} ctok_tables;
int ctok_create_from_tables(const ctok_tables* tables, ctok** out);
void ctok_destroy(ctok* tok);

/* Tokenizer.vocab_size                      src/bindings/tokenizer.rs:271-274 -> mod.rs:856-858 */
uint64_t ctok_vocab_size(const ctok* tok);
/* Tokenizer.token_to_id(token)              src/bindings/tokenizer.rs:276-278 -> mod.rs:860-862 */
int ctok_token_to_id(const ctok* tok, const char* token, size_t len, uint32_t* id);
/* Tokenizer.id_to_token(id)                 src/bindings/tokenizer.rs:280-282 -> mod.rs:864-866
 * Writes up to cap bytes and sets *len to the full length (call again with a larger buffer). */
int ctok_id_to_token(const ctok* tok, uint32_t id, char* buf, size_t cap, size_t* len);
/* Tokenizer.special_tokens (dict)           src/bindings/tokenizer.rs:284-289 */
uint64_t ctok_num_special_tokens(const ctok* tok);
int ctok_special_token(const ctok* tok, uint64_t i, char* buf, size_t cap, size_t* len, uint32_t* id);

/* Diagnostics of the added-token split (src/huggingface/mod.rs:566-675).  The reference tries
 * every added token on every pre-tokenized word; tokens that provably never occur inside one
 * GPT2_PATTERN piece (e.g. "<|endoftext|>", which the regex always cuts apart) cannot change
 * the result and are left out of the device tables at load.
 *   ctok_num_piece_added_tokens: how many added tokens the encode kernels split on (0 = the
 *     fast paths without the split run);
 *   ctok_piece_can_contain: 1 if the raw byte string can occur inside one piece (the load-time
 *     predicate; conservative: 1 unless provably impossible), 0 if not, < 0 on error. */
uint64_t ctok_num_piece_added_tokens(const ctok* tok);
int ctok_piece_can_contain(const uint8_t* raw, size_t len);

/* Execution / measurement options for one encode call. */
typedef struct ctok_exec {
  int device;       /* HIP device ordinal the work runs on                              */
  void* stream;     /* hipStream_t to order the work on; NULL = the library's stream      */
  uint32_t flags;   /* CTOK_F_* */
  /* ctok_encode_batch (host buffers) only; zero = defaults: */
  const int* devices;     /* shard the batch over these devices (contiguous doc ranges balanced by
                             bytes, one host thread each, no collective); NULL = { device }      */
  int n_devices;
  uint32_t chunk_mb;      /* pipeline chunk: MiB of text per H2D -> encode -> D2H step (0 = 64)  */
  uint32_t host_threads;  /* host threads widening 16-bit ids per device (0 = auto)            */
} ctok_exec;

#define CTOK_F_TIMING 1u  /* record per-kernel HIP events (fills ctok_stats.ms_*) */

typedef struct ctok_stats {
  double ms_total;        /* wall time of the call (host clock)                        */
  double ms_device;       /* first kernel start -> last kernel end (HIP events)        */
  double ms_pretok;       /* normalise check + doc bitmap + pre-tokenizer/routing      */
  double ms_bpe_short;    /* merge passes of pieces <= 64 bytes (k_segment's end -> the last one's end) */
  double ms_bpe_long;     /* wait for the side stream (long-piece tiers) after them         */
  double ms_emit;         /* tile token scan + id emission + tok_off                   */
  double ms_h2d, ms_d2h;  /* host-buffer copies (ctok_encode_batch only)               */
  uint64_t bytes_in;      /* raw UTF-8 bytes of the batch                              */
  uint64_t bytes_norm;    /* bytes after normalisation / prefix space                  */
  uint64_t docs, pieces, long_pieces, tokens, nfc_docs;  /* nfc_docs: documents NFC-normalised (a superset
                                                          of those NFC changes: flagged per 64-byte word) */
  double ms_segment;      /* k_segment (from k_tilefirst's end): piece starts + probes/routing */
  double ms_bpe_lo;       /* k_bpe_short (from k_segment's end): pieces of <= 16 bytes     */
  double ms_bpe_hi;       /* k_bpe_mid<2>: pieces of 17..32 bytes (on the side stream: the time it adds after k_bpe_short) */
  uint64_t class_bytes[4];  /* text bytes merged per length class (<= 8, 9..16, 17..32, 33..64 B) */
  uint64_t class_ids[4];    /* ids produced per length class                             */
  double ms_bpe_med;      /* 33..64-byte pieces (k_bpe_mid<3> main instance or k_bpe_sparse), after k_bpe_short */
  uint64_t workspace_bytes; /* device workspace held by the device for this tokenizer's calls */
  uint64_t long_rounds;     /* merge rounds of the long-piece wave tiers (<= 4096 B pieces), summed over pieces */
} ctok_stats;

/* Upper bound on the ids of a batch whose docs total `n_bytes` bytes (ids <= 3*bytes + docs:
 * NFC can grow UTF-8 at most 3x, add_prefix_space adds one byte per doc). */
uint64_t ctok_ids_bound(const ctok* tok, uint64_t n_bytes, uint64_t n_docs);

/* Tokenizer.encode_batch(texts) on host buffers   src/bindings/tokenizer.rs:207-210
 *   -> HuggingFaceTokenizer::encode_batch          src/huggingface/mod.rs:694-696
 * The batch moves in chunks (exec->chunk_mb, ramped from 1/8 of it at both ends) copied straight
 * from / to the caller's buffers: the H2D copy of the next chunk and the D2H copy of the previous
 * one overlap the kernels of the current one (ids cross the link as 16-bit values when every id
 * the tokenizer can emit is < 2^16, widened into `ids` by host threads).  With
 * exec->devices, each device encodes its own byte-balanced doc range the same way (the
 * reference's rayon par_iter over docs, one GPU per range instead of one core per doc).
 * utf8[doc_off[d] .. doc_off[d+1]) is document d (valid UTF-8, doc_off[0] == 0,
 * non-decreasing).  On success ids[tok_off[d] .. tok_off[d+1]) are its token ids.
 * Tokenizer.encode(text) is the n_docs == 1 case (src/bindings/tokenizer.rs:203-205). */
int ctok_encode_batch(const ctok* tok, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                      uint32_t* ids, uint64_t ids_cap, uint64_t* tok_off,
                      const ctok_exec* exec, ctok_stats* stats);

/* Same, with every buffer already resident in HBM of exec->device (device pointers) and the
 * work ordered on exec->stream.  n_bytes = doc_off[n_docs] (passed so the host need not read
 * device memory).  *n_tokens_out (host) receives the total number of ids written. */
int ctok_encode_batch_device(const ctok* tok, const uint8_t* d_utf8, const uint64_t* d_doc_off,
                             uint64_t n_docs, uint64_t n_bytes, uint32_t* d_ids, uint64_t ids_cap,
                             uint64_t* d_tok_off, uint64_t* n_tokens_out,
                             const ctok_exec* exec, ctok_stats* stats);

/* ---------------------------------------------------------------- decode (ids -> UTF-8 text)
 * decode_impl, src/huggingface/mod.rs:710-747, per document:
 *   - skip_special_tokens drops ids whose model.vocab string is a special added token (:716-726);
 *   - ids are looked up in model.vocab only (Vocab::get_token, src/vocab.rs:91-93); unknown ids
 *     are dropped;
 *   - the ByteLevel decoder maps the tokens' chars back to bytes, then from_utf8_lossy
 *     (src/decoders.rs:94-119); an unknown decoder type joins the raw token strings
 *     (BpeTokenizer::decode, src/bpe.rs:170-176); other decoders -> CTOK_E_UNSUPPORTED;
 *   - clean_up_tokenization_spaces: 15 replaces, then split_whitespace joined by ' ' (:749-767). */
#define CTOK_D_SKIP_SPECIAL 1u  /* skip_special_tokens                          */
#define CTOK_D_CLEANUP 2u       /* clean_up_tokenization_spaces (the default on) */

typedef struct ctok_decode_stats {
  double ms_total;        /* wall time of the call (host clock)                          */
  double ms_device;       /* ms_len + ms_gather + ms_clean                                */
  double ms_len;          /* offsets check + decoded bytes per id chunk + scan (HIP events) */
  double ms_gather;       /* id -> bytes gather                                           */
  double ms_clean;        /* lossy UTF-8 + clean-up: mark, count, scan, write            */
  double ms_h2d, ms_d2h;  /* host-buffer copies (ctok_decode_batch only)                  */
  uint64_t ids, docs;
  uint64_t bytes_raw;     /* decoded bytes before lossy UTF-8 / clean-up                  */
  uint64_t bytes_out;     /* output bytes                                                 */
  uint32_t direct;        /* 1: no clean-up and all bytes ASCII, the gather wrote the output */
} ctok_decode_stats;

/* Tokenizer.decode_batch_with_options(batch, skip_special_tokens, clean_up_tokenization_spaces)
 *   src/bindings/tokenizer.rs:231-238 -> src/huggingface/mod.rs:777-785; decode_batch (:226-228
 *   -> :771-773), decode (:212-214), decode_with_options (:217-224) and batch_decode (:656-663)
 *   are the same call with options CTOK_D_CLEANUP and/or one document.
 * ids[tok_off[d] .. tok_off[d+1]) are document d's ids (tok_off[0] == 0, non-decreasing).  On
 * success out[out_off[d] .. out_off[d+1]) is its UTF-8 text.  out_cap too small -> CTOK_E_CAPACITY
 * with out_off filled (out_off[n_docs] = bytes needed). */
int ctok_decode_batch(const ctok* tok, const uint32_t* ids, const uint64_t* tok_off, uint64_t n_docs,
                      uint32_t options, uint8_t* out, uint64_t out_cap, uint64_t* out_off,
                      const ctok_exec* exec, ctok_decode_stats* stats);

/* Same, with ids / tok_off / out / out_off resident in HBM of exec->device and the work ordered
 * on exec->stream; n_ids = tok_off[n_docs].  *n_bytes_out receives the output size (also on
 * CTOK_E_CAPACITY, when out_cap is too small and nothing is written). */
int ctok_decode_batch_device(const ctok* tok, const uint32_t* d_ids, const uint64_t* d_tok_off, uint64_t n_docs,
                             uint64_t n_ids, uint32_t options, uint8_t* d_out, uint64_t out_cap,
                             uint64_t* d_out_off, uint64_t* n_bytes_out, const ctok_exec* exec,
                             ctok_decode_stats* stats);

/* ------------------------------------------------- padded batch encode (Encoding rows as arrays)
 * Tokenizer.__call__ / encode_batch_with_padding / encode_batch_to_encoding / encode_to_encoding
 * (src/bindings/tokenizer.rs:46-201, :298-371 -> src/huggingface/mod.rs:340-545,
 * src/encoding.rs:45-253), computed on the GPU as [rows, width] u32 arrays:
 *   - CTOK_P_ADD_SPECIAL: the encode_to_encoding flavour -- words go to BPE with no added-token
 *     split (mod.rs:395-420), the post-processor's process(ids, None) is applied (a pair is
 *     merged first, so the *single* template wraps both sequences, mod.rs:365-376), the masks
 *     are extended by the added count and special tokens are marked (mod.rs:378-387).
 *     Without it: Encoding::from_ids over Tokenizer.encode's ids (tokenizer.rs:88-97).
 *   - CTOK_P_PAIRS: docs 2r and 2r+1 form row r; the second sequence's ids get type id 1.
 *   - CTOK_P_TRUNCATE: rows cut to max_length (Encoding::truncate keeps the first max_length).
 *   - CTOK_P_PAD_LONGEST / CTOK_P_PAD_TO_MAX: pad (Encoding::pad) to the longest row / to
 *     max_length, on the left with CTOK_P_PAD_LEFT; pad id = opts->pad_id with CTOK_P_PAD_ID,
 *     else the reference's choice (special "[PAD]", else "<pad>", else 0).  Padding cells:
 *     attention 0, type 0, special 1.  A row longer than the target is not cut.
 * Row r occupies ids[r*width .. r*width + row_len[r]); cells past row_len hold padding values.
 * attention / type_ids / special_mask may be NULL.  cap = elements available in each array;
 * rows * width > cap -> CTOK_E_CAPACITY with *width_out and row_len filled.  A template that
 * drops ids (the reference's usize underflow at mod.rs:378) -> CTOK_E_PANIC. */
#define CTOK_P_ADD_SPECIAL 1u
#define CTOK_P_PAIRS 2u
#define CTOK_P_TRUNCATE 4u
#define CTOK_P_PAD_LONGEST 8u
#define CTOK_P_PAD_TO_MAX 16u
#define CTOK_P_PAD_LEFT 32u
#define CTOK_P_PAD_ID 64u
#define CTOK_P_NO_POSTPROCESS 128u  /* with CTOK_P_ADD_SPECIAL: skip the post-processor (ids, marks) */

typedef struct ctok_pad_opts {
  uint32_t flags;       /* CTOK_P_* */
  uint32_t pad_id;      /* with CTOK_P_PAD_ID */
  uint64_t max_length;  /* CTOK_P_TRUNCATE limit and CTOK_P_PAD_TO_MAX target */
} ctok_pad_opts;

int ctok_encode_padded(const ctok* tok, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                       const ctok_pad_opts* opts, uint32_t* ids, uint32_t* attention_mask, uint32_t* type_ids,
                       uint32_t* special_mask, uint64_t cap, uint64_t* row_len, uint64_t* width_out,
                       const ctok_exec* exec, ctok_stats* stats);
/* Same on HBM-resident buffers (device pointers, work on exec->stream); n_bytes = doc_off[n_docs]. */
int ctok_encode_padded_device(const ctok* tok, const uint8_t* d_utf8, const uint64_t* d_doc_off, uint64_t n_docs,
                              uint64_t n_bytes, const ctok_pad_opts* opts, uint32_t* d_ids, uint32_t* d_attention,
                              uint32_t* d_type_ids, uint32_t* d_special, uint64_t cap, uint64_t* d_row_len,
                              uint64_t* width_out, const ctok_exec* exec, ctok_stats* stats);
/* The model_max_length used when max_length is not given (512 for from_file / from_str,
 * src/huggingface/mod.rs:243-245) and the pad id the reference picks (mod.rs:500-504). */
uint64_t ctok_model_max_length(const ctok* tok);
uint32_t ctok_pad_id(const ctok* tok);
/* The post-processor as applied by the padded encode: *n_items items (at most cap written), each
 * CTOK_PP_SEQUENCE (the sequence's ids, "$A") or a special id; *n_items = -1 without one. */
#define CTOK_PP_SEQUENCE 0xFFFFFFFFu
int ctok_post_processor(const ctok* tok, uint32_t* items, uint64_t cap, int64_t* n_items);
/* Tokenizer.num_special_tokens_to_add(is_pair)  src/bindings/tokenizer.rs:248-251 -> mod.rs:915-932 */
uint64_t ctok_num_special_tokens_to_add(const ctok* tok, int is_pair);

/* Offsets and word ids of encode_to_encoding, before the post-processor
 * (encode_single_to_encoding + pre_tokenize_with_offsets, src/huggingface/mod.rs:395-480; replaces
 * the per-text Encoding.offsets / Encoding.word_ids of src/bindings/encoding.rs).  Each document
 * is encoded on the GPU without the added-token split (ids[tok_off[d] .. tok_off[d+1])); token k's
 * byte range in its document is offsets[2k] .. offsets[2k+1] and word_ids[k] is the index of its
 * pre-tokenized word.  The reference's approximations are kept (each word found with str::find
 * from the previous word's end, falling back to the word's byte-level length; each token's range
 * is its token string's byte length, clipped to the word).  A fallback that ends inside a UTF-8
 * character makes the reference panic on the next word: CTOK_E_PANIC.  cap too small ->
 * CTOK_E_CAPACITY with tok_off filled. */
int ctok_encode_offsets(const ctok* tok, const uint8_t* utf8, const uint64_t* doc_off, uint64_t n_docs,
                        uint32_t* ids, uint64_t* offsets, uint32_t* word_ids, uint64_t cap, uint64_t* tok_off,
                        const ctok_exec* exec);

/* Number of HIP devices visible to the library (0 when none; encode calls then fail with
 * CTOK_E_DEVICE -- there is no CPU fallback). */
int ctok_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* CTOK_H */
