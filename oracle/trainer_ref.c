/* TEST / MEASUREMENT INFRASTRUCTURE -- not product code.
 *
 * A C restatement of the reference trainer's per-merge work, used as the CPU baseline of the
 * trainer timing (tools/trainer_timing.py) and checked against oracle/trainer_ref.py
 * (tests/test_trainer_cpu.py):
 *
 *   apply_merge_incremental   /root/reference/src/trainer.rs:519-588
 *     words.par_iter_mut(): each word rescanned left to right, a HashMap of pair deltas per
 *     word (here: one per thread, the same sums), the merged occurrences' freqs summed;
 *     then the deltas aggregated into pair_freqs, token_freqs updated (saturating), and
 *     pair_freqs.retain(v > 0) over the whole map;
 *   build_heap                /root/reference/src/trainer.rs:369-405 (every 100 merges, :419)
 *     an f32 INL score per live pair and a binary heap of them (O(pairs) heapify).
 *
 * The merges themselves (which pair, which new id) are an input: the sequence a training run
 * chose (the GPU trainer's, or oracle/trainer_ref.py's), so this times the reference's cost per
 * merge on the same words without restating its heap-pop tie rules.  Threads: the caller's count
 * (rayon's default pool: every CPU of the affinity mask).
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* open-addressing map (u64 key -> i64), keys != ~0 */
typedef struct {
  uint64_t* k;
  int64_t* v;
  uint64_t cap, n;
} pmap;

static const uint64_t kEmpty = ~0ull;

static uint64_t hmix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

static void pm_init(pmap* m, uint64_t cap) {
  uint64_t c = 16;
  while (c < 2 * cap) c <<= 1;
  m->cap = c;
  m->n = 0;
  m->k = (uint64_t*)malloc(c * 8);
  m->v = (int64_t*)malloc(c * 8);
  memset(m->k, 0xFF, c * 8);
}

static void pm_free(pmap* m) {
  free(m->k);
  free(m->v);
}

static void pm_add(pmap* m, uint64_t key, int64_t d);

static void pm_grow(pmap* m) {
  pmap n;
  pm_init(&n, m->cap);
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->k[i] != kEmpty) pm_add(&n, m->k[i], m->v[i]);
  pm_free(m);
  *m = n;
}

static void pm_add(pmap* m, uint64_t key, int64_t d) {
  if (2 * (m->n + 1) > m->cap) pm_grow(m);
  uint64_t h = hmix(key) & (m->cap - 1);
  while (m->k[h] != kEmpty && m->k[h] != key) h = (h + 1) & (m->cap - 1);
  if (m->k[h] == kEmpty) {
    m->k[h] = key;
    m->v[h] = 0;
    m->n++;
  }
  m->v[h] += d;
}

/* pair_freqs.remove(&pair): its count set to 0 -- the same map after the retain(v > 0) that ends
 * the merge (deltas that re-insert the pair are non-positive then as in the reference) */
static void pm_zero(pmap* m, uint64_t key) {
  uint64_t h = hmix(key) & (m->cap - 1);
  while (m->k[h] != kEmpty && m->k[h] != key) h = (h + 1) & (m->cap - 1);
  if (m->k[h] == key) m->v[h] = 0;
}

/* retain(v > 0): rebuilt in place (the reference walks every bucket of its map) */
static void pm_retain_positive(pmap* m) {
  pmap n;
  pm_init(&n, m->n);
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->k[i] != kEmpty && m->v[i] > 0) pm_add(&n, m->k[i], m->v[i]);
  pm_free(m);
  *m = n;
}

typedef struct {
  uint32_t n_words;
  const uint64_t* off; /* word w: toks[off[w] .. off[w] + len[w]) */
  uint32_t* toks;
  uint32_t* len;
  const uint64_t* freq;
} words_t;

typedef struct {
  words_t* W;
  uint32_t w0, w1, a, b, nid;
  pmap deltas;
  uint64_t tf;
} job_t;

static void* apply_range(void* p) {
  job_t* j = (job_t*)p;
  words_t* W = j->W;
  j->tf = 0;
  for (uint32_t w = j->w0; w < j->w1; w++) {
    uint32_t* t = W->toks + W->off[w];
    uint32_t n = W->len[w];
    const int64_t f = (int64_t)W->freq[w];
    uint32_t i = 0;
    while (n >= 2 && i < n - 1) {
      if (t[i] == j->a && t[i + 1] == j->b) {
        if (i > 0) pm_add(&j->deltas, ((uint64_t)t[i - 1] << 32) | j->a, -f);
        if (i + 2 < n) pm_add(&j->deltas, ((uint64_t)j->b << 32) | t[i + 2], -f);
        t[i] = j->nid;
        memmove(t + i + 1, t + i + 2, (size_t)(n - i - 2) * 4);
        n--;
        if (i > 0) pm_add(&j->deltas, ((uint64_t)t[i - 1] << 32) | j->nid, f);
        if (i + 1 < n) pm_add(&j->deltas, ((uint64_t)j->nid << 32) | t[i + 1], f);
        j->tf += (uint64_t)f;
      } else {
        i++;
      }
    }
    W->len[w] = n;
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* f32 INL score of a pair (build_heap, trainer.rs:380-399), one rounding per operation */
static float inl_score(int64_t f, float fa, float fb, float va, float vb, float mu, float alpha, float beta_c,
                       float vmax, float gate) {
  float ea = fa - mu, eb = fb - mu;
  float van = fminf(fmaxf(alpha * va - beta_c * ea, -vmax), vmax);
  float vbn = fminf(fmaxf(alpha * vb - beta_c * eb, -vmax), vmax);
  return (float)f - gate * (van + vbn);
}

static void sift_down(float* h, uint64_t n, uint64_t i) {
  for (;;) {
    uint64_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && h[l] > h[m]) m = l;
    if (r < n && h[r] > h[m]) m = r;
    if (m == i) return;
    float x = h[i];
    h[i] = h[m];
    h[m] = x;
    i = m;
  }
}

/* Apply `n_merges` merges (a[k], b[k]) -> nid[k] to the words, with the reference's per-merge
 * bookkeeping; pair_freqs starts as the words' adjacent-pair histogram (compute_initial_pairs),
 * token_freqs[id] (ids < n_ids) as given.  Times the merges (apply + aggregate + retain) and the
 * heap rebuilds (every 100 merges) separately.  Returns the number of live pairs at the end. */
uint64_t trm_run(uint32_t n_words, const uint64_t* off, uint32_t* toks, uint32_t* len, const uint64_t* freq,
                 uint32_t n_merges, const uint32_t* ma, const uint32_t* mb, const uint32_t* mnid, uint64_t* token_freqs,
                 uint32_t n_ids, int threads, double* secs_merges, double* secs_heap) {
  words_t W = {n_words, off, toks, len, freq};
  pmap pf;
  pm_init(&pf, 1 << 16);
  for (uint32_t w = 0; w < n_words; w++)
    for (uint32_t i = 0; i + 1 < len[w]; i++)
      pm_add(&pf, ((uint64_t)toks[off[w] + i] << 32) | toks[off[w] + i + 1], (int64_t)freq[w]);
  if (threads < 1) threads = 1;
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  float* velocity = (float*)calloc(n_ids, sizeof(float));
  float* heap = NULL;
  double tm = 0, th_ = 0;
  for (uint32_t k = 0; k < n_merges; k++) {
    if (k % 100 == 0) {  /* build_heap: scores of every live pair, heapified */
      double t0 = now_s();
      uint64_t total = 0;
      for (uint32_t i = 0; i < n_ids; i++) total += token_freqs[i];
      const float mu = 0.01f * (float)total, beta_c = fmaxf(fminf(0.3f, 2.0f), 0.0f);
      free(heap);
      heap = (float*)malloc((pf.n + 1) * sizeof(float));
      uint64_t n = 0;
      for (uint64_t i = 0; i < pf.cap; i++) {
        if (pf.k[i] == kEmpty || pf.v[i] <= 0) continue;
        uint32_t a = (uint32_t)(pf.k[i] >> 32), b = (uint32_t)pf.k[i];
        heap[n++] = inl_score(pf.v[i], (float)token_freqs[a < n_ids ? a : 0], (float)token_freqs[b < n_ids ? b : 0],
                              velocity[a < n_ids ? a : 0], velocity[b < n_ids ? b : 0], mu, 0.9f, beta_c, 10.0f, 0.5f);
      }
      for (uint64_t i = n / 2; i-- > 0;) sift_down(heap, n, i);
      th_ += now_s() - t0;
    }
    double t0 = now_s();
    const uint32_t a = ma[k], b = mb[k], nid = mnid[k];
    pm_zero(&pf, ((uint64_t)a << 32) | b);
    const uint32_t per = (n_words + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; t++) {
      job_t* j = &jobs[t];
      j->W = &W;
      j->w0 = (uint32_t)t * per < n_words ? (uint32_t)t * per : n_words;
      j->w1 = j->w0 + per < n_words ? j->w0 + per : n_words;
      j->a = a;
      j->b = b;
      j->nid = nid;
      pm_init(&j->deltas, 64);
      if (threads > 1) pthread_create(&th[t], NULL, apply_range, j);
      else apply_range(j);
    }
    uint64_t tf = 0;
    for (int t = 0; t < threads; t++) {
      if (threads > 1) pthread_join(th[t], NULL);
      job_t* j = &jobs[t];
      tf += j->tf;
      for (uint64_t i = 0; i < j->deltas.cap; i++)
        if (j->deltas.k[i] != kEmpty) pm_add(&pf, j->deltas.k[i], j->deltas.v[i]);
      pm_free(&j->deltas);
    }
    if (a < n_ids) token_freqs[a] = token_freqs[a] > tf ? token_freqs[a] - tf : 0;
    if (b < n_ids) token_freqs[b] = token_freqs[b] > tf ? token_freqs[b] - tf : 0;
    if (nid < n_ids) {
      token_freqs[nid] = tf;
      velocity[nid] = (velocity[a < n_ids ? a : 0] + velocity[b < n_ids ? b : 0]) / 2.0f;
    }
    pm_retain_positive(&pf);
    tm += now_s() - t0;
  }
  free(heap);
  free(velocity);
  free(jobs);
  free(th);
  uint64_t live = pf.n;
  pm_free(&pf);
  if (secs_merges) *secs_merges = tm;
  if (secs_heap) *secs_heap = th_;
  return live;
}
