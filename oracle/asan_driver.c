/* ORACLE -- test infrastructure only (tests/test_oracle_asan.py).  A driver
 * for the C restatement built with -fsanitize=address,undefined: tokenises
 * the sentences of a raw file (bytes + int64 offsets) at max_tok with
 * nthreads threads and writes the sparse ids and counts, so the sanitizer
 * runs over the golden inputs (tokenizer_oracle.c's orc_tok_run, the
 * restatement of lddl/dask/bert/pretrain.py:79-80's tokenizer call).
 *   asan_driver VOCAB TABLE BYTES OFFS N_SENT MAX_TOK NTHREADS OUT_IDS OUT_NTOK */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void *orc_tok_create(const char *vocab_path, const char *table_path);
void orc_tok_destroy(void *h);
int orc_tok_run(void *h, const uint8_t *bytes, const int64_t *sent_off, int64_t n_sent, int max_tok,
                int32_t *out_ids, int32_t *out_ntok, int nthreads);

static void *slurp(const char *path, long *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void *p = malloc(*n > 0 ? (size_t)*n : 1);
  if (*n > 0 && fread(p, 1, (size_t)*n, f) != (size_t)*n) { free(p); p = NULL; }
  fclose(f);
  return p;
}

int main(int argc, char **argv) {
  if (argc != 10) { fprintf(stderr, "usage: asan_driver VOCAB TABLE BYTES OFFS N MAXTOK NTH IDS NTOK\n"); return 2; }
  long nb = 0, no = 0;
  uint8_t *bytes = slurp(argv[3], &nb);
  int64_t *off = slurp(argv[4], &no);
  const int64_t n = atoll(argv[5]);
  if (!bytes || !off || no != (long)((n + 1) * 8)) { fprintf(stderr, "bad input files\n"); return 2; }
  void *h = orc_tok_create(argv[1], argv[2]);
  if (!h) { fprintf(stderr, "cannot load vocab / table\n"); return 2; }
  const int64_t span = off[n] - off[0];
  int32_t *ids = calloc(span > 0 ? (size_t)span : 1, sizeof(int32_t));
  int32_t *ntok = calloc(n > 0 ? (size_t)n : 1, sizeof(int32_t));
  orc_tok_run(h, bytes, off, n, atoi(argv[6]), ids, ntok, atoi(argv[7]));
  FILE *fi = fopen(argv[8], "wb"), *fn = fopen(argv[9], "wb");
  if (!fi || !fn) return 2;
  fwrite(ids, sizeof(int32_t), span > 0 ? (size_t)span : 0, fi);
  fwrite(ntok, sizeof(int32_t), (size_t)n, fn);
  fclose(fi);
  fclose(fn);
  orc_tok_destroy(h);
  free(ids);
  free(ntok);
  free(bytes);
  free(off);
  return 0;
}
