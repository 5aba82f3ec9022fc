/*
 * Host sentence splitter of the preprocessor CLI (lddl_amd/preprocess.py):
 * the rule-based stand-in for NLTK Punkt (_rule_split) together with
 * split_id_text (readers.py:142-147) and split_records' strip / drop-empty
 * step (pretrain.py:82-97 _to_document), over the records' raw UTF-8 bytes.
 * It produces exactly what the Python path produces from the same records;
 * tests/test_split_native.py compares the two.  Python semantics are kept
 * code point by code point:
 *   whitespace        str.isspace (== re's \s)     table bit 0
 *   next char starts  str.isupper / str.isdigit    bits 1 / 2
 *   one-letter word   len(c.lower()) == 1 and c.lower().isalpha()   bit 3
 *   c.lower() is ASCII only for ASCII and U+212A (KELVIN SIGN -> 'k')
 * The tables come from the running Python (unicodedata of its version).
 * Invalid UTF-8 (which the Python path's strict decode rejects) returns -2
 * with the record's index, so the caller re-runs that chunk in Python.
 * Plain C, no GPU: the CLI's forked split workers load it.
 */
#include <stdint.h>
#include <string.h>

enum { P_SPACE = 1, P_UPPER = 2, P_DIGIT = 4, P_ALPHA1 = 8 };

static const char *const ABBREV[] = {"mr",  "mrs",  "ms",  "dr",  "prof", "sr",  "jr",     "st",  "vs",  "etc", "e.g",
                                     "i.e", "inc",  "ltd", "co",  "corp", "jan", "feb",    "mar", "apr", "jun", "jul",
                                     "aug", "sep",  "sept", "oct", "nov",  "dec", "no",     "fig", "al",  "approx",
                                     "dept", "est", "gen", "gov", "lt",   "mt",  "rev",    "sgt", "u.s", "u.k"};

/* strict UTF-8 decode of the code point at s[i] (i < n): its length in *len,
 * -1 when invalid (overlong, surrogate, > U+10FFFF, truncated) */
static int32_t dec(const uint8_t *s, int64_t i, int64_t n, int *len) {
  const uint32_t b = s[i];
  if (b < 0x80) {
    *len = 1;
    return (int32_t)b;
  }
  int k;
  uint32_t c, lo;
  if (b >= 0xC2 && b <= 0xDF) {
    k = 1;
    c = b & 0x1F;
    lo = 0x80;
  } else if (b >= 0xE0 && b <= 0xEF) {
    k = 2;
    c = b & 0x0F;
    lo = 0x800;
  } else if (b >= 0xF0 && b <= 0xF4) {
    k = 3;
    c = b & 0x07;
    lo = 0x10000;
  } else {
    return -1;
  }
  for (int j = 1; j <= k; ++j) {
    if (i + j >= n) return -1;
    const uint32_t x = s[i + j];
    if ((x & 0xC0) != 0x80) return -1;
    c = (c << 6) | (x & 0x3F);
  }
  if (c < lo || c > 0x10FFFF || (c >= 0xD800 && c <= 0xDFFF)) return -1;
  *len = k + 1;
  return (int32_t)c;
}

static inline int prop(const uint8_t *tab, int32_t c) { return tab[c]; }

static inline uint64_t load8(const uint8_t *p) {
  uint64_t x;
  memcpy(&x, p, 8);
  return x;
}
#define ONES 0x0101010101010101ull
#define HIGHS 0x8080808080808080ull
/* some byte of x equals b */
static inline int has_byte(uint64_t x, uint8_t b) {
  const uint64_t y = x ^ (ONES * b);
  return ((y - ONES) & ~y & HIGHS) != 0;
}

/* strict UTF-8 over [i, n): 0, or -1 at the first invalid sequence */
static int valid(const uint8_t *s, int64_t i, int64_t n) {
  int len;
  while (i < n) {
    if (i + 8 <= n && !(load8(s + i) & HIGHS)) {
      i += 8;
      continue;
    }
    if (s[i] < 0x80) {
      ++i;
      continue;
    }
    if (dec(s, i, n, &len) < 0) return -1;
    i += len;
  }
  return 0;
}

/* start of the code point ending just before byte i (i > b0) */
static int64_t back(const uint8_t *s, int64_t i, int64_t b0) {
  --i;
  while (i > b0 && (s[i] & 0xC0) == 0x80) --i;
  return i;
}

static int is_close(uint8_t b) { return b == '"' || b == '\'' || b == ')' || b == ']'; }
static int is_strip(uint8_t b) { return b == '(' || b == '"' || b == '\'' || b == '['; }

/* the word before a '.' break is an abbreviation or a one-letter initial */
static int no_break_word(const uint8_t *s, int64_t a, int64_t e, const uint8_t *tab) {
  while (a < e && is_strip(s[a])) ++a;
  while (e > a && is_strip(s[e - 1])) --e;
  if (a >= e) return 0;
  /* one code point: its lowercase is one alphabetic character */
  int len;
  const int32_t c0 = dec(s, a, e, &len);
  if (c0 >= 0 && a + len == e) return (prop(tab, c0) & P_ALPHA1) != 0;
  /* the lowered word, when it is ASCII */
  char w[8];
  int m = 0;
  for (int64_t i = a; i < e;) {
    const int32_t c = dec(s, i, e, &len);
    if (c < 0 || m >= 7) return 0;
    if (c < 0x80) w[m++] = (char)(c >= 'A' && c <= 'Z' ? c + 32 : c);
    else if (c == 0x212A) w[m++] = 'k';
    else return 0;
    i += len;
  }
  w[m] = 0;
  for (unsigned k = 0; k < sizeof(ABBREV) / sizeof(ABBREV[0]); ++k)
    if (strcmp(w, ABBREV[k]) == 0) return 1;
  return 0;
}

typedef struct {
  uint8_t *out;
  int64_t out_n, out_cap;
  int64_t *sent_off;
  int64_t n_sent, sent_cap;
} Sink;

/* bytes [a, e) stripped of whitespace at both ends; appended unless empty */
static int emit(Sink *k, const uint8_t *s, int64_t a, int64_t e, const uint8_t *tab) {
  int len;
  while (a < e) {
    const int32_t c = dec(s, a, e, &len);
    if (c < 0) return -2;
    if (!(prop(tab, c) & P_SPACE)) break;
    a += len;
  }
  while (e > a) {
    const int64_t p = back(s, e, a);
    const int32_t c = dec(s, p, e, &len);
    if (c < 0) return -2;
    if (!(prop(tab, c) & P_SPACE)) break;
    e = p;
  }
  if (a >= e) return 0;
  if (k->out_n + (e - a) > k->out_cap || k->n_sent + 1 > k->sent_cap) return -3;
  memcpy(k->out + k->out_n, s + a, (size_t)(e - a));
  k->out_n += e - a;
  k->sent_off[++k->n_sent] = k->out_n;
  return 0;
}

/* _rule_split over body [b0, b1) + split_records' strip / drop */
static int split_body(Sink *k, const uint8_t *s, int64_t b0, int64_t b1, const uint8_t *tab) {
  int64_t start = b0, pos = b0;
  int len, rc;
  for (;;) {
    /* the next match of [.!?]+["')\]]*\s+ at or after pos (finditer) */
    int64_t i = pos, ms = -1, me = -1;
    while (i < b1) {
      if (i + 8 <= b1) {  /* 8 bytes at a time to the next [.!?] */
        const uint64_t x = load8(s + i);
        if (!has_byte(x, '.') && !has_byte(x, '!') && !has_byte(x, '?')) {
          i += 8;
          continue;
        }
      }
      const uint8_t b = s[i];
      if (b != '.' && b != '!' && b != '?') {
        ++i;
        continue;
      }
      int64_t j = i;
      while (j < b1 && (s[j] == '.' || s[j] == '!' || s[j] == '?')) ++j;
      int64_t q = j;
      while (q < b1 && is_close(s[q])) ++q;
      int64_t w = q;
      while (w < b1) {
        const int32_t c = dec(s, w, b1, &len);
        if (c < 0) return -2;
        if (!(prop(tab, c) & P_SPACE)) break;
        w += len;
      }
      if (w > q) {
        ms = i;
        me = w;
        break;
      }
      i = j;  /* (positions inside the run fail the same way) */
    }
    if (ms < 0 || me >= b1) break;
    pos = me;
    const int32_t nx = dec(s, me, b1, &len);
    if (nx < 0) return -2;
    if (!((prop(tab, nx) & (P_UPPER | P_DIGIT)) || nx == '"' || nx == '\'' || nx == '(' || nx == '[')) continue;
    if (s[ms] == '.') {
      /* the last whitespace-separated word of [start, ms) */
      int64_t e = ms;
      while (e > start) {
        const int64_t p = back(s, e, start);
        const int32_t c = dec(s, p, e, &len);
        if (c < 0) return -2;
        if (!(prop(tab, c) & P_SPACE)) break;
        e = p;
      }
      int64_t a = e;
      while (a > start) {
        const int64_t p = back(s, a, start);
        const int32_t c = dec(s, p, a, &len);
        if (c < 0) return -2;
        if (prop(tab, c) & P_SPACE) break;
        a = p;
      }
      if (no_break_word(s, a, e, tab)) continue;
    }
    if ((rc = emit(k, s, start, me, tab))) return rc;
    start = me;
  }
  return emit(k, s, start, b1, tab);
}

/* Records r = buf[rec_off[r], rec_off[r+1]): "<id><ws><body>" each.  Writes
 * the sentences back to back into out (out_cap bytes), out_sent_off[0..n]
 * (out_sent_off[0] = 0; sent_cap entries after it), out_doc_sent_off[r+1]
 * = sentences after record r, out_id[2r], [2r+1] = the id's byte range in buf.
 * Returns the number of sentences, -2 (invalid UTF-8; *bad = the record) or
 * -3 (capacity). */
int64_t lddl_split_rules(const uint8_t *buf, const int64_t *rec_off, int64_t n_rec, const uint8_t *tab,
                         uint8_t *out, int64_t out_cap, int64_t *out_sent_off, int64_t sent_cap,
                         int64_t *out_doc_sent_off, int64_t *out_id, int64_t *bad) {
  Sink k = {out, 0, out_cap, out_sent_off, 0, sent_cap};
  out_sent_off[0] = 0;
  out_doc_sent_off[0] = 0;
  for (int64_t r = 0; r < n_rec; ++r) {
    const int64_t r0 = rec_off[r], r1 = rec_off[r + 1];
    int64_t i = r0;
    int len = 0;
    int32_t c = 0;
    while (i < r1) {
      c = dec(buf, i, r1, &len);
      if (c < 0) {
        *bad = r;
        return -2;
      }
      if (prop(tab, c) & P_SPACE) break;
      i += len;
    }
    out_id[2 * r] = r0;
    out_id[2 * r + 1] = i;
    const int64_t b0 = i < r1 ? i + len : r1;  /* raw[i + 1:]: one code point skipped */
    /* the rest of the record must decode too (the Python path decodes it whole) */
    if (valid(buf, b0, r1) < 0) {
      *bad = r;
      return -2;
    }
    const int rc = split_body(&k, buf, b0, r1, tab);
    if (rc) {
      *bad = r;
      return rc;
    }
    out_doc_sent_off[r + 1] = k.n_sent;
  }
  return k.n_sent;
}

/* The line spans of buf[0, n) as readers._line_spans makes them (terminators
 * excluded; universal newlines: CR LF, lone CR and lone LF each end a line;
 * crlf_only: CR LF alone; no final line after a last terminator).  Returns
 * the number of lines; starts / ends are written when it is <= cap (a first
 * call with cap 0 counts them). */
int64_t lddl_line_spans(const uint8_t *buf, int64_t n, int32_t crlf_only, int64_t *starts, int64_t *ends,
                        int64_t cap) {
  int64_t m = 0, a = 0, p = 0;
#define LINE(s_, e_)              \
  do {                            \
    if (m < cap) {                \
      starts[m] = (s_);           \
      ends[m] = (e_);             \
    }                             \
    ++m;                          \
  } while (0)
  /* one streaming pass: memchr to the next LF; in universal mode the bytes
   * before it (still in cache) are checked for CR (a lone CR ends a line;
   * CR LF ends one line) */
  while (p < n) {
    const uint8_t *f = memchr(buf + p, '\n', (size_t)(n - p));
    const int64_t t = f ? (int64_t)(f - buf) : n;
    if (crlf_only) {
      if (!f) break;
      p = t + 1;
      if (t == 0 || buf[t - 1] != '\r') continue;
      LINE(a, t - 1);
      a = t + 1;
      continue;
    }
    int crlf = 0;
    const uint8_t *r = memchr(buf + p, '\r', (size_t)(t - p));
    while (r) {
      const int64_t c = (int64_t)(r - buf);
      LINE(a, c);
      a = c + 1;
      if (c + 1 == t) {  /* CR LF: one terminator */
        crlf = 1;
        break;
      }
      r = memchr(buf + a, '\r', (size_t)(t - a));
    }
    if (!f) break;
    if (!crlf) LINE(a, t);
    a = t + 1;
    p = t + 1;
  }
  if (a < n) LINE(a, n);
#undef LINE
  return m;
}
