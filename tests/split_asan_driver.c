/* Test driver (tests/test_split_asan.py): lddl_amd/host/split_rules.c built
 * with AddressSanitizer + UndefinedBehaviorSanitizer.  Buffers are sized
 * exactly (no slack) so any out-of-bounds access is reported.
 *   split_asan_driver TAB BUF REC_OFF N_REC OUT
 * TAB: the code point property table (0x110000 bytes); BUF: the records'
 * bytes; REC_OFF: int64[N_REC + 1].  Writes OUT.split (int64 rc, int64 bad,
 * then on success out bytes, sent_off[rc + 1], doc_sent_off[N_REC + 1],
 * id ranges[2 N_REC]) and OUT.lines (per mode universal / CR LF only: int64
 * m, starts[m], ends[m]). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t lddl_split_rules(const uint8_t *buf, const int64_t *rec_off, int64_t n_rec, const uint8_t *tab,
                         uint8_t *out, int64_t out_cap, int64_t *out_sent_off, int64_t sent_cap,
                         int64_t *out_doc_sent_off, int64_t *out_id, int64_t *bad);
int64_t lddl_line_spans(const uint8_t *buf, int64_t n, int32_t crlf_only, int64_t *starts, int64_t *ends,
                        int64_t cap);

static void *slurp(const char *path, int64_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  *n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void *p = malloc(*n > 0 ? (size_t)*n : 1);
  if (*n > 0 && fread(p, 1, (size_t)*n, f) != (size_t)*n) exit(2);
  fclose(f);
  return p;
}

static void put(FILE *f, const void *p, size_t n) {
  if (n && fwrite(p, 1, n, f) != n) exit(2);
}

int main(int argc, char **argv) {
  if (argc != 6) return 2;
  int64_t ntab, nbuf, noff;
  uint8_t *tab = slurp(argv[1], &ntab);
  uint8_t *buf = slurp(argv[2], &nbuf);
  int64_t *rec_off = slurp(argv[3], &noff);
  const int64_t n_rec = atoll(argv[4]);
  if (ntab != 0x110000 || noff != 8 * (n_rec + 1) || rec_off[n_rec] != nbuf) return 2;
  char path[4096];
  snprintf(path, sizeof path, "%s.split", argv[5]);
  FILE *fo = fopen(path, "wb");
  /* out never exceeds the input bytes; sentences: a first call at a small
   * capacity (exercising the -3 return), then at one per input byte */
  uint8_t *out = malloc(nbuf > 0 ? (size_t)nbuf : 1);
  int64_t *doc = malloc(sizeof(int64_t) * (size_t)(n_rec + 1));
  int64_t *ids = malloc(sizeof(int64_t) * (size_t)(2 * n_rec + 1));
  int64_t bad = -1, rc, cap = 1;
  for (;;) {
    int64_t *soff = malloc(sizeof(int64_t) * (size_t)(cap + 1));
    rc = lddl_split_rules(buf, rec_off, n_rec, tab, out, nbuf, soff, cap, doc, ids, &bad);
    if (rc >= 0) {
      put(fo, &rc, 8);
      put(fo, &bad, 8);
      put(fo, out, (size_t)soff[rc]);
      put(fo, soff, 8 * (size_t)(rc + 1));
      put(fo, doc, 8 * (size_t)(n_rec + 1));
      put(fo, ids, 8 * (size_t)(2 * n_rec));
    }
    free(soff);
    if (rc != -3 || cap >= nbuf + 1) break;
    cap = cap * 8 < nbuf + 1 ? cap * 8 : nbuf + 1;  /* (non-empty sentences: at most one per byte) */
  }
  if (rc < 0) {
    put(fo, &rc, 8);
    put(fo, &bad, 8);
  }
  fclose(fo);
  snprintf(path, sizeof path, "%s.lines", argv[5]);
  fo = fopen(path, "wb");
  for (int32_t mode = 0; mode < 2; ++mode) {
    const int64_t m = lddl_line_spans(buf, nbuf, mode, NULL, NULL, 0);
    int64_t *s = malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
    int64_t *e = malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
    if (lddl_line_spans(buf, nbuf, mode, s, e, m) != m) return 3;
    put(fo, &m, 8);
    put(fo, s, 8 * (size_t)m);
    put(fo, e, 8 * (size_t)m);
    free(s);
    free(e);
  }
  fclose(fo);
  free(out);
  free(doc);
  free(ids);
  free(tab);
  free(buf);
  free(rec_off);
  return 0;
}
