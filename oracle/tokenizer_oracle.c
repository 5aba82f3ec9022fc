/*
 * ORACLE -- test infrastructure only.  Never linked into or called by the
 * product path (lddl_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so.
 *
 * Plain-C CPU restatement of the tokenizer the reference calls per sentence:
 *   lddl/dask/bert/pretrain.py:79-80   tokenizer.tokenize(s, max_length=512,
 *                                      truncation=True)
 *   lddl/dask/bert/pretrain.py:584-587 transformers.BertTokenizerFast(vocab)
 *   lddl/dask/bert/pretrain_codebert.py:123-124 (same call, code lines)
 * The arithmetic lives in the third-party HF `tokenizers` crate (pinned here:
 * 0.22.2, the wheel in this image; the reference pins only transformers
 * 4.16.2 in setup.py:55).  Published algorithm restated:
 *   1. added-token split: leftmost literal match of [PAD] [UNK] [CLS] [SEP]
 *      [MASK] on the RAW text (normalized=false added tokens);
 *   2. BertNormalizer on every other segment: clean_text, CJK padding,
 *      NFD + drop Mn (strip_accents follows lowercase), per-char lowercase.
 *      Per-code-point outputs come from lddl_amd/data/unicode_table.bin
 *      (generated from tokenizers by tools/gen_unicode_table.py); NFD
 *      canonical reordering of surviving ccc>0 chars is applied per run;
 *   3. BertPreTokenizer: split on whitespace, isolate punctuation;
 *   4. WordPiece(unk=[UNK], prefix=##, max_input_chars_per_word=100),
 *      greedy longest-match-first, whole word -> [UNK] on any failure;
 *   5. transformers 4.16.2 truncation: keep the first max_tok tokens.
 * Parity of this restatement is pinned by tests/golden/tok_*.npz and
 * tests/golden/normalize_fuzz.json (both produced by tokenizers 0.22.2).
 *
 * Output convention (shared with the HIP path, include/lddl_amd.h):
 *   sentence s's ids are written at out_ids[sent_off[s] - sent_off[0] ...],
 *   out_ntok[s] = number of ids (<= max_tok).  #tokens <= #bytes always holds
 *   (checked over every code point by the table generator).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define KIND_IDENT 0
#define KIND_MAP 1
#define KIND_DROP_T 2
#define KIND_DROP_D 3
#define KIND_MULTI 4
#define CLS_OTHER 0
#define CLS_SPACE 1
#define CLS_ISOLATE 2

typedef struct {
  char *str;
  int len;
  int id;
} vent_t;

typedef struct {
  uint16_t top[0x1100];
  uint32_t *pages;
  uint32_t (*multi)[4];
  int n_pages, n_multi;
  vent_t *vocab;
  int n_vocab;
  int *slots; /* open addressing, -1 empty */
  uint64_t cap;
  int special_id[5];
  int unk_id;
} orc_tok_t;

static const char *SPECIAL[5] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};

static uint64_t fnv1a(const char *s, int n) {
  uint64_t h = 1469598103934665603ULL;
  for (int i = 0; i < n; ++i) {
    h ^= (unsigned char)s[i];
    h *= 1099511628211ULL;
  }
  return h;
}

static int vocab_find(const orc_tok_t *t, const char *s, int n) {
  uint64_t h = fnv1a(s, n) & (t->cap - 1);
  for (;;) {
    int v = t->slots[h];
    if (v < 0) return -1;
    if (t->vocab[v].len == n && memcmp(t->vocab[v].str, s, n) == 0) return t->vocab[v].id;
    h = (h + 1) & (t->cap - 1);
  }
}

void orc_tok_destroy(void *h) {
  orc_tok_t *t = (orc_tok_t *)h;
  if (!t) return;
  for (int i = 0; i < t->n_vocab; ++i) free(t->vocab[i].str);
  free(t->vocab);
  free(t->slots);
  free(t->pages);
  free(t->multi);
  free(t);
}

void *orc_tok_create(const char *vocab_path, const char *table_path) {
  orc_tok_t *t = (orc_tok_t *)calloc(1, sizeof(orc_tok_t));
  FILE *f = fopen(table_path, "rb");
  if (!f) { free(t); return NULL; }
  char magic[8];
  uint32_t hdr[3];
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "LDDLUNI1", 8) || fread(hdr, 4, 3, f) != 3) {
    fclose(f); free(t); return NULL;
  }
  t->n_pages = hdr[0];
  t->n_multi = hdr[1];
  t->pages = (uint32_t *)malloc((size_t)t->n_pages * 256 * 4);
  t->multi = malloc((size_t)t->n_multi * 16);
  if (fread(t->top, 2, 0x1100, f) != 0x1100 ||
      fread(t->pages, 4, (size_t)t->n_pages * 256, f) != (size_t)t->n_pages * 256 ||
      fread(t->multi, 16, t->n_multi, f) != (size_t)t->n_multi) {
    fclose(f); orc_tok_destroy(t); return NULL;
  }
  fclose(f);

  /* vocab.txt: line i -> id i, trailing whitespace trimmed */
  f = fopen(vocab_path, "rb");
  if (!f) { orc_tok_destroy(t); return NULL; }
  int cap = 1024;
  t->vocab = (vent_t *)malloc(sizeof(vent_t) * cap);
  char line[4096];
  while (fgets(line, sizeof line, f)) {
    int n = (int)strlen(line);
    while (n > 0 && (line[n - 1] == '\n' || line[n - 1] == '\r' || line[n - 1] == ' ' || line[n - 1] == '\t')) --n;
    if (t->n_vocab == cap) { cap *= 2; t->vocab = (vent_t *)realloc(t->vocab, sizeof(vent_t) * cap); }
    t->vocab[t->n_vocab].str = (char *)malloc(n + 1);
    memcpy(t->vocab[t->n_vocab].str, line, n);
    t->vocab[t->n_vocab].str[n] = 0;
    t->vocab[t->n_vocab].len = n;
    t->vocab[t->n_vocab].id = t->n_vocab;
    t->n_vocab++;
  }
  fclose(f);
  t->cap = 1;
  while (t->cap < (uint64_t)t->n_vocab * 2) t->cap <<= 1;
  t->slots = (int *)malloc(sizeof(int) * t->cap);
  for (uint64_t i = 0; i < t->cap; ++i) t->slots[i] = -1;
  for (int i = 0; i < t->n_vocab; ++i) {
    uint64_t h = fnv1a(t->vocab[i].str, t->vocab[i].len) & (t->cap - 1);
    for (;;) {
      int v = t->slots[h];
      if (v < 0) { t->slots[h] = i; break; }
      if (t->vocab[v].len == t->vocab[i].len && !memcmp(t->vocab[v].str, t->vocab[i].str, t->vocab[i].len)) {
        t->slots[h] = i; /* duplicate line: last id wins */
        break;
      }
      h = (h + 1) & (t->cap - 1);
    }
  }
  for (int k = 0; k < 5; ++k) {
    t->special_id[k] = vocab_find(t, SPECIAL[k], (int)strlen(SPECIAL[k]));
    if (t->special_id[k] < 0) { orc_tok_destroy(t); return NULL; }
  }
  t->unk_id = t->special_id[1];
  return t;
}

int orc_tok_vocab_size(void *h) { return ((orc_tok_t *)h)->n_vocab; }
int orc_tok_special_id(void *h, int k) { return ((orc_tok_t *)h)->special_id[k]; }

/* ---------------- per-sentence restatement ---------------- */

typedef struct {
  uint32_t cp;
  int rank;
  int cls;
  int delim; /* removed char that breaks a ccc run */
} item_t;

static int utf8_decode(const uint8_t *s, int64_t n, int64_t i, uint32_t *cp) {
  uint8_t b = s[i];
  if (b < 0x80) { *cp = b; return 1; }
  int len = (b >= 0xF0) ? 4 : (b >= 0xE0) ? 3 : 2;
  uint32_t c = b & (0x3F >> (len - 1));
  for (int k = 1; k < len && i + k < n; ++k) c = (c << 6) | (s[i + k] & 0x3F);
  *cp = c;
  return len;
}

static int utf8_encode(uint32_t c, char *o) {
  if (c < 0x80) { o[0] = (char)c; return 1; }
  if (c < 0x800) { o[0] = (char)(0xC0 | (c >> 6)); o[1] = (char)(0x80 | (c & 0x3F)); return 2; }
  if (c < 0x10000) {
    o[0] = (char)(0xE0 | (c >> 12)); o[1] = (char)(0x80 | ((c >> 6) & 0x3F)); o[2] = (char)(0x80 | (c & 0x3F));
    return 3;
  }
  o[0] = (char)(0xF0 | (c >> 18)); o[1] = (char)(0x80 | ((c >> 12) & 0x3F));
  o[2] = (char)(0x80 | ((c >> 6) & 0x3F)); o[3] = (char)(0x80 | (c & 0x3F));
  return 4;
}

typedef struct {
  item_t *it;
  int n, cap;
  char *wb; /* word bytes */
  int wcap;
} scratch_t;

static void push_item(scratch_t *sc, uint32_t cp, int rank, int cls, int delim) {
  if (sc->n == sc->cap) { sc->cap = sc->cap ? sc->cap * 2 : 256; sc->it = (item_t *)realloc(sc->it, sizeof(item_t) * sc->cap); }
  item_t *x = &sc->it[sc->n++];
  x->cp = cp; x->rank = rank; x->cls = cls; x->delim = delim;
}

/* normalise raw segment [b,e) into items (delimiters kept as markers) */
static void normalize_segment(const orc_tok_t *t, const uint8_t *s, int64_t b, int64_t e, scratch_t *sc) {
  sc->n = 0;
  int64_t i = b;
  while (i < e) {
    uint32_t cp;
    i += utf8_decode(s, e, i, &cp);
    if (cp > 0x10FFFF) cp = 0xFFFD;
    uint32_t ent = t->pages[(size_t)t->top[cp >> 8] * 256 + (cp & 255)];
    int kind = ent >> 26, cls = (ent >> 24) & 3, rank = (ent >> 21) & 7;
    switch (kind) {
      case KIND_IDENT: push_item(sc, cp, rank, cls, 0); break;
      case KIND_MAP: push_item(sc, ent & 0x1FFFFF, rank, cls, 0); break;
      case KIND_DROP_T: break;
      case KIND_DROP_D: push_item(sc, 0, 0, CLS_OTHER, 1); break;
      default: {
        const uint32_t *m = t->multi[ent & 0x1FFFFF];
        for (uint32_t k = 0; k < m[0]; ++k) {
          uint32_t x = m[1 + k];
          push_item(sc, x & 0x1FFFFF, (x >> 21) & 7, (x >> 24) & 3, 0);
        }
      }
    }
  }
  /* canonical reordering: stable sort each maximal run of rank>0 items */
  for (int a = 0; a < sc->n;) {
    if (sc->it[a].rank == 0) { ++a; continue; }
    int z = a;
    while (z < sc->n && sc->it[z].rank > 0) ++z;
    for (int p = a + 1; p < z; ++p) { /* insertion sort, stable */
      item_t x = sc->it[p];
      int q = p - 1;
      while (q >= a && sc->it[q].rank > x.rank) { sc->it[q + 1] = sc->it[q]; --q; }
      sc->it[q + 1] = x;
    }
    a = z;
  }
}

typedef struct {
  int32_t *out;
  int n, max;
} emit_t;

static inline void emit(emit_t *o, int id) {
  if (o->n < o->max) o->out[o->n] = id;
  o->n++;
}

static void wordpiece(const orc_tok_t *t, const item_t *w, int nchar, scratch_t *sc, emit_t *o) {
  if (nchar > 100) { emit(o, t->unk_id); return; }
  if (sc->wcap < nchar * 4 + 8) { sc->wcap = nchar * 4 + 8; sc->wb = (char *)realloc(sc->wb, sc->wcap); }
  /* byte offset of each char in the word (and the end) */
  int off[101];
  int nb = 0;
  for (int k = 0; k < nchar; ++k) { off[k] = nb; nb += utf8_encode(w[k].cp, sc->wb + nb); }
  off[nchar] = nb;
  int mark = o->n;
  int start = 0;
  char cand[512];
  while (start < nchar) {
    int end = nchar, found = -1;
    while (start < end) {
      int len = off[end] - off[start], n;
      if (start > 0) { cand[0] = '#'; cand[1] = '#'; memcpy(cand + 2, sc->wb + off[start], len); n = len + 2; }
      else { memcpy(cand, sc->wb + off[start], len); n = len; }
      found = vocab_find(t, cand, n);
      if (found >= 0) break;
      --end;
    }
    if (found < 0) { o->n = mark; emit(o, t->unk_id); return; }
    emit(o, found);
    start = end;
  }
}

/* BertPreTokenizer over the normalised items: CLS_SPACE ends a word,
 * CLS_ISOLATE is a word of its own; delimiter markers are not chars. */
typedef void (*word_fn)(const orc_tok_t *t, const item_t *w, int nchar, scratch_t *sc, void *arg);

static void split_words(const orc_tok_t *t, scratch_t *sc, word_fn fn, void *arg) {
  item_t *word = NULL;
  int wn = 0, wcap = 0;
  for (int k = 0; k < sc->n; ++k) {
    const item_t *x = &sc->it[k];
    if (x->delim) continue;
    if (x->cls == CLS_OTHER) {
      if (wn == wcap) { wcap = wcap ? wcap * 2 : 64; word = (item_t *)realloc(word, sizeof(item_t) * wcap); }
      word[wn++] = *x;
      continue;
    }
    if (wn > 0) fn(t, word, wn, sc, arg);
    wn = 0;
    if (x->cls == CLS_ISOLATE) fn(t, x, 1, sc, arg);
  }
  if (wn > 0) fn(t, word, wn, sc, arg);
  free(word);
}

static void wp_cb(const orc_tok_t *t, const item_t *w, int nchar, scratch_t *sc, void *arg) {
  wordpiece(t, w, nchar, sc, (emit_t *)arg);
}

static void tokenize_text(const orc_tok_t *t, const uint8_t *s, int64_t b, int64_t e, scratch_t *sc, emit_t *o) {
  normalize_segment(t, s, b, e, sc);
  split_words(t, sc, wp_cb, o);
}

static int match_special(const uint8_t *s, int64_t i, int64_t e, int *which) {
  if (s[i] != '[') return 0;
  for (int k = 0; k < 5; ++k) {
    int n = (int)strlen(SPECIAL[k]);
    if (i + n <= e && memcmp(s + i, SPECIAL[k], n) == 0) { *which = k; return n; }
  }
  return 0;
}

int orc_tok_sentence(const orc_tok_t *t, const uint8_t *s, int64_t b, int64_t e, int max_tok, int32_t *out, scratch_t *sc) {
  emit_t o = {out, 0, max_tok};
  int64_t seg = b;
  for (int64_t i = b; i < e;) {
    int which;
    int n = match_special(s, i, e, &which);
    if (n) {
      if (i > seg) tokenize_text(t, s, seg, i, sc, &o);
      emit(&o, t->special_id[which]);
      i += n;
      seg = i;
    } else {
      ++i;
    }
  }
  if (e > seg) tokenize_text(t, s, seg, e, sc, &o);
  return o.n < max_tok ? o.n : max_tok;
}

typedef struct {
  const orc_tok_t *t;
  const uint8_t *bytes;
  const int64_t *sent_off;
  int64_t lo, hi;
  int max_tok;
  int32_t *out_ids;
  int32_t *out_ntok;
} job_t;

static void *worker(void *p) {
  job_t *j = (job_t *)p;
  scratch_t sc = {0};
  int64_t base = j->sent_off[0];
  for (int64_t s = j->lo; s < j->hi; ++s) {
    int64_t b = j->sent_off[s], e = j->sent_off[s + 1];
    j->out_ntok[s] = orc_tok_sentence(j->t, j->bytes, b, e, j->max_tok, j->out_ids + (b - base), &sc);
  }
  free(sc.it);
  free(sc.wb);
  return NULL;
}

/* Tokenise n_sent sentences with nthreads host threads (sparse output). */
int orc_tok_run(void *h, const uint8_t *bytes, const int64_t *sent_off, int64_t n_sent, int max_tok,
                int32_t *out_ids, int32_t *out_ntok, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t th[256];
  job_t jobs[256];
  if (nthreads > 256) nthreads = 256;
  int64_t per = (n_sent + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    jobs[k] = (job_t){(orc_tok_t *)h, bytes, sent_off, k * per, (k + 1) * per, max_tok, out_ids, out_ntok};
    if (jobs[k].lo > n_sent) jobs[k].lo = n_sent;
    if (jobs[k].hi > n_sent) jobs[k].hi = n_sent;
    if (nthreads == 1) worker(&jobs[k]);
    else pthread_create(&th[k], NULL, worker, &jobs[k]);
  }
  if (nthreads > 1)
    for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
  return 0;
}

/* Normalise + pre-tokenise one raw string (no special-token split); words
 * are written as UTF-8 separated by '\n' (for the fuzz fixture). */
typedef struct { char *out; int64_t o, cap; int err; } words_t;

static void words_cb(const orc_tok_t *t, const item_t *w, int nchar, scratch_t *sc, void *arg) {
  (void)t; (void)sc;
  words_t *x = (words_t *)arg;
  for (int k = 0; k < nchar; ++k) {
    char buf[8];
    int m = utf8_encode(w[k].cp, buf);
    if (x->o + m + 1 > x->cap) { x->err = 1; return; }
    memcpy(x->out + x->o, buf, m);
    x->o += m;
  }
  x->out[x->o++] = '\n';
}

int64_t orc_words(void *h, const uint8_t *s, int64_t n, char *out, int64_t cap) {
  orc_tok_t *t = (orc_tok_t *)h;
  scratch_t sc = {0};
  words_t x = {out, 0, cap, 0};
  normalize_segment(t, s, 0, n, &sc);
  split_words(t, &sc, words_cb, &x);
  free(sc.it);
  free(sc.wb);
  return x.err ? -1 : x.o;
}
