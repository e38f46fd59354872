/* ctok_trainer.h -- C ABI of the INL-BPE trainer with GPU pair counting.
 *
 * Drop-in for the reference's PyO3 class `complexity_tokenizer.Trainer`
 * (Complexity-ML/complexity-tokenizer v0.3.3, src/bindings/trainers.rs:10-92, registered at
 * src/lib.rs:50) over `InlBpeTrainer` (src/trainer.rs).  Word counting pre-tokenizes on the GPU
 * (NFC + ByteLevel, the encode path's k_segment) and counts words on the host; the pair histogram
 * (compute_initial_pairs, src/trainer.rs:341-367) and every merge's pass over the words with its
 * pair-count deltas (apply_merge_incremental, :522-590) run on the GPU; the INL-scored heap
 * (build_heap / learn_merges_heap, :369-520) runs on the host in f32 exactly as the reference.
 *
 * The reference leaves two orders to randomly seeded hash iteration; this library fixes them
 * (alphabet ids in ascending code point order; equal heap scores in ascending
 * (token_a, token_b) byte order, then ids).  Errors: 0 or a negative CTOK_E_* code (ctok.h),
 * ctok_last_error() holds the message.  A ctok_trainer* is not thread-safe.
 */
#ifndef CTOK_TRAINER_H
#define CTOK_TRAINER_H

#include <stddef.h>
#include <stdint.h>

#include "ctok.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ctok_trainer ctok_trainer;

/* TrainerConfig (src/trainer.rs:66-110); Trainer(...) defaults at src/bindings/trainers.rs:19-27. */
typedef struct ctok_trainer_config {
  uint64_t vocab_size;        /* 32000 */
  uint32_t min_frequency;     /* 2 */
  uint64_t min_word_length;   /* 1 */
  float inl_alpha;            /* 0.9 */
  float inl_beta;             /* 0.3 */
  float inl_gate;             /* 0.5 */
  float inl_mu_target;        /* 0.01 */
  float inl_velocity_max;     /* 10.0 */
  float inl_beta_max;         /* 2.0 */
  /* special tokens: n_special UTF-8 strings, token i = special[special_off[i] .. special_off[i+1]) */
  const char* special;
  const uint64_t* special_off;
  uint64_t n_special;
  int device;                 /* HIP device of the pair counting */
} ctok_trainer_config;

/* Trainer(vocab_size, min_frequency, special_tokens, ...)   src/bindings/trainers.rs:28-55 */
int ctok_trainer_create(const ctok_trainer_config* cfg, ctok_trainer** out);
void ctok_trainer_destroy(ctok_trainer* tr);

/* Word counting of n_texts UTF-8 texts (text i = utf8[off[i] .. off[i+1])), each NFC-normalised
 * and ByteLevel pre-tokenized; words of >= min_word_length chars are counted.
 *   into_accumulator = 1: Trainer.count_batch   (src/trainer.rs:207-220, the accumulator)
 *   into_accumulator = 0: the word counts of train_from_iterator / train(files) (:245-285),
 *                         kept until the next ctok_trainer_train(tr, 0) */
int ctok_trainer_count(ctok_trainer* tr, const uint8_t* utf8, const uint64_t* off, uint64_t n_texts,
                       int into_accumulator);

/* Drop the counts of ctok_trainer_count(tr, ..., accumulator).  train(files) counts its files in
 * blocks as it reads them; when a later line is not UTF-8 it drops what it counted, as the
 * reference's count_words returns the io::Error before any count is kept (src/trainer.rs:265-285). */
int ctok_trainer_clear_counts(ctok_trainer* tr, int accumulator);

/* from_accumulator = 1: Trainer.finish_training (src/trainer.rs:223-229); 0: the training step of
 * train_from_iterator / train(files) on the counts of ctok_trainer_count(..., 0).  Both drop words
 * below min_frequency, then train_from_word_freqs (:231-243). */
int ctok_trainer_train(ctok_trainer* tr, int from_accumulator);

/* train_from_word_freqs on words given directly: word i = raw (unmapped) bytes
 * words[word_off[i] .. word_off[i+1]) with frequency freqs[i]. */
int ctok_trainer_train_words(ctok_trainer* tr, const uint8_t* words, const uint64_t* word_off, const uint32_t* freqs,
                             uint64_t n_words);

/* Trainer.vocab_size / num_merges getters   src/bindings/trainers.rs:83-91 */
uint64_t ctok_trainer_vocab_size(const ctok_trainer* tr);
uint64_t ctok_trainer_num_merges(const ctok_trainer* tr);

/* The tokenizer.json of Trainer.save (src/trainer.rs:600-645): writes up to cap bytes to buf and
 * sets *len to the full length.  ctok_trainer_save writes it to path. */
int ctok_trainer_json(const ctok_trainer* tr, char* buf, size_t cap, size_t* len);
int ctok_trainer_save(const ctok_trainer* tr, const char* path);

/* The pair histogram of the last training's compute_initial_pairs, sorted by (a, b):
 * writes up to cap entries and sets *n to the number of pairs. */
int ctok_trainer_initial_pairs(const ctok_trainer* tr, uint32_t* a, uint32_t* b, int64_t* count, uint64_t cap,
                               uint64_t* n);

/* Milliseconds of the last training spent in GPU pair counting / merge application / host heap. */
int ctok_trainer_timing(const ctok_trainer* tr, double* ms_pairs, double* ms_merges, double* ms_heap);

#ifdef __cplusplus
}
#endif

#endif /* CTOK_TRAINER_H */
