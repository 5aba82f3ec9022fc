/*
 * lddl_amd -- C-ABI of the MI355X (gfx950) preprocessing hot path.
 *
 * The reference (alvin-zyl/LDDL) is pure Python; its hot path sits behind
 * three seams, each replaced here by an entry point of liblddl_amd.so:
 *
 *   lddl_create / lddl_destroy
 *       replaces transformers.BertTokenizerFast(vocab_file)
 *       (lddl/dask/bert/pretrain.py:584-587, pretrain_codebert.py:617 --
 *       the latter substituted by WordPiece over codebert_52000/vocab.txt).
 *   lddl_tokenize
 *       replaces the per-sentence tokenizer.tokenize(s, max_length=512,
 *       truncation=True) of _get_documents._to_document
 *       (pretrain.py:79-80, :82-95) and _get_code_pairs (pretrain_codebert.py:
 *       123-124), batched over every sentence of a shard.
 *   lddl_pack_bert / lddl_pack_codebert / lddl_materialize / lddl_masked_lm
 *       replace _get_pairs._to_partition_pairs (pretrain.py:386-402 with
 *       create_pairs_from_document :241-365 and, with --masking,
 *       create_masked_lm_predictions :182-238; pretrain_codebert.py:460-477
 *       with :343-442) and the binned writer's grouping
 *       (binning.py:63-93 _to_dataframe_binned).  A pack call writes its
 *       result into a caller-owned lddl_pack (lddl_pack_new; NULL = the
 *       ctx's own) that the post-pack calls then name explicitly.
 *   lddl_bin
 *       replaces _to_dataframe_binned's grouping (binning.py:63-93) on its
 *       own, for any column of row lengths.
 *
 * Conventions: every pointer named d_* is a DEVICE pointer on the ctx's
 * device; work is enqueued on `stream` (a hipStream_t, NULL = default) and is
 * asynchronous.  Return value 0 = ok, < 0 = LDDL_E* (message: lddl_last_error,
 * thread-local).  One call at a time per ctx (the ctx owns scratch).
 * Input text must be valid UTF-8 (Python str.encode output).
 */
#ifndef LDDL_AMD_H_
#define LDDL_AMD_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDDL_EINVAL -1
#define LDDL_EIO -2
#define LDDL_EFORMAT -3
#define LDDL_ENOMEM -4
#define LDDL_EHIP -5
#define LDDL_ECAPACITY -6
/* pretrain_codebert.py:421 _truncate_seq(code, max_num - len(doc)) with a
 * negative budget raises IndexError in the reference; reported as this code */
#define LDDL_EINDEX -7
/* pretrain.py:330-331 / pretrain_codebert.py:423 assert len(...) >= 1 */
#define LDDL_EASSERT -8

typedef struct lddl_ctx lddl_ctx;
/* The result of one lddl_pack_bert / lddl_pack_codebert call: pair records,
 * their shuffled and binned order, per-partition counts, the masking draws.
 * lddl_materialize / lddl_row_spans / lddl_masked_lm[_spans] / lddl_row_docs
 * read the result they are given, so several results can be live at once
 * (e.g. one shard set packed while the previous one is written).  Every call
 * taking a `pack` accepts NULL = the ctx's own result.  A pack result's
 * device buffers grow on demand and are reused by the next pack into it;
 * a failed pack leaves it empty (post-pack calls return LDDL_EINVAL). */
typedef struct lddl_pack lddl_pack;

const char *lddl_last_error(void);

/* vocab.txt: line i -> id i (reference: BertTokenizerFast(vocab_file)).
 * table_path: lddl_amd/data/unicode_table.bin. */
int lddl_create(const char *vocab_path, const char *table_path, int device, lddl_ctx **out);
void lddl_destroy(lddl_ctx *ctx);
int lddl_vocab_size(const lddl_ctx *ctx);
/* ids of [PAD] [UNK] [CLS] [SEP] [MASK] */
int lddl_special_ids(const lddl_ctx *ctx, int32_t out[5]);
/* NUL-terminated vocab entry `id` into buf; returns its length */
int lddl_vocab_token(const lddl_ctx *ctx, int32_t id, char *buf, int64_t cap);

/* Tokenise n_sent sentences (bytes [d_sent_off[s], d_sent_off[s+1])) into
 * the dense CSR layout: sentence s's ids are
 * d_out_ids[d_out_tok_off[s] .. d_out_tok_off[s+1]), d_out_ntok[s] = their
 * count = min(#tokens, max_tok), d_out_tok_off[n_sent] = the total
 * (d_out_tok_off: n_sent + 1 entries).  out_cap = entries of d_out_ids: ids
 * past it are not written, the offsets are still complete, so a caller that
 * finds d_out_tok_off[n_sent] > out_cap calls again with a larger buffer;
 * out_cap >= nbytes always suffices (#tokens <= #bytes).  nbytes must be >=
 * d_sent_off[n_sent] - d_sent_off[0]; 1 <= max_tok <= 65534.  d_bytes:
 * 4-byte aligned.  lddl_pack_* / lddl_materialize read d_out_ids with 16-B
 * loads: keep it 16-B aligned with 16 entries of padding past the total. */
int lddl_tokenize(lddl_ctx *ctx, const uint8_t *d_bytes, int64_t nbytes, const int64_t *d_sent_off,
                  int64_t n_sent, int32_t max_tok, uint16_t *d_out_ids, int64_t out_cap, int32_t *d_out_ntok,
                  int64_t *d_out_tok_off, void *stream);

/* Per-kernel timing of lddl_tokenize (diagnostics / bench): with timing on,
 * every call records HIP events around its kernels on the call's stream;
 * lddl_tokenize_stats (synchronises on them) returns out[0..5] = scan,
 * WordPiece and finish (serial-path tiles + counts + offset scan + dense
 * expand) milliseconds of the last call (summed over its segments), the
 * number of WordPiece records it ran, the number of segments (launches of
 * each kernel) and the number of tiles sent to the serial path. */
int lddl_set_timing(lddl_ctx *ctx, int on);
int lddl_tokenize_stats(lddl_ctx *ctx, double *out, int n);

/* With on != 0, every following lddl_tokenize also records which sentences
 * hold a [CLS] / [SEP] token (pretrain.py:187-190 excludes those tokens
 * from the masking candidates); a masked lddl_pack_bert over the same
 * d_out_ids / d_out_ntok buffers then reuses the flags instead of a pass
 * over the ids.  Off by default (the unmasked path does not need them). */
int lddl_set_special_flags(lddl_ctx *ctx, int on);

/* The tokenizer algorithm of the following lddl_tokenize calls (A/B and
 * tests; every algorithm gives identical ids): 5 = the split tokenizer (the
 * default), 6 = the lane tokenizer, 0 = every tile through the exact serial
 * path.  An algorithm that does not model the loaded tables falls back to 0;
 * so does 6 on a ctx created without LDDL_TOKENIZE_ALGO=6 or
 * LDDL_WP_ALGO=trie in the environment (its trie is built only then).
 * *out_algo (may be NULL) receives the one selected.  Scratch is kept across
 * a switch; each call allocates what its algorithm reads. */
int lddl_set_tokenize_algo(lddl_ctx *ctx, int algo, int *out_algo);

/* A new, empty pack result on ctx's device (free with lddl_pack_free, before
 * or after the ctx).  lddl_pack_rows: #rows of its last successful pack, -1
 * when none. */
int lddl_pack_new(lddl_ctx *ctx, lddl_pack **out);
void lddl_pack_free(lddl_pack *pack);
int lddl_pack_rows(const lddl_pack *pack, int64_t *out_npairs);

/* Pack every partition of a tokenised shard set into `pack`.
 * Partition p = docs [d_part_doc_off[p], d_part_doc_off[p+1]); doc d =
 * sentences [d_doc_sent_off[d], d_doc_sent_off[d+1]); d_ids / d_ntok /
 * d_tok_off / d_sent_off are lddl_tokenize's output / input (d_ids may be
 * NULL unless masking; all of them must stay live until lddl_materialize;
 * every d_ntok count <= 65535, as any lddl_tokenize output with max_tok <=
 * 65535 -- the packers keep the counts as u16).  Partition p is packed exactly like the reference's
 * _to_partition_pairs (pretrain.py:386-402) after random.seed(seed + p):
 * duplicate_factor passes of create_pairs_from_document (:241-365), then
 * random.shuffle, then (bin_size > 0) the stable bin grouping of
 * binning.py:63-93.  Synchronises the stream once and returns
 * out_totals[4] = {#pairs, #tokens (with [CLS]/[SEP]), nbins, #masked}.
 * masking != 0: static MLM masking, create_masked_lm_predictions
 * (:182-238) with vocab_words = the vocab file's tokens in file order
 * (target_seq_length <= 1024); the rows are then written by
 * lddl_materialize and masked by lddl_masked_lm. */
int lddl_pack_bert(lddl_ctx *ctx, lddl_pack *pack, const uint16_t *d_ids, const int32_t *d_ntok, const int64_t *d_tok_off,
                   const int64_t *d_sent_off, int64_t n_sent, const int64_t *d_doc_sent_off, int64_t n_doc,
                   const int64_t *d_part_doc_off, int64_t n_part, int32_t target_seq_length, double short_seq_prob,
                   int32_t duplicate_factor, int32_t masking, double masked_lm_ratio, uint64_t seed, int32_t bin_size,
                   int64_t *out_totals,
                   void *stream);

/* CodeBERT docstring/code packing (pretrain_codebert.py:343-442, :460-477).
 * Doc d's first d_doc_nseg_doc[d] sentences are its docstring segments, the
 * rest its code segments (one per source line, pretrain_codebert.py:126-159). */
int lddl_pack_codebert(lddl_ctx *ctx, lddl_pack *pack, const int32_t *d_ntok, const int64_t *d_tok_off, const int64_t *d_sent_off,
                       int64_t n_sent, const int64_t *d_doc_sent_off, const int32_t *d_doc_nseg_doc, int64_t n_doc,
                       const int64_t *d_part_doc_off, int64_t n_part, int32_t target_seq_length,
                       double short_seq_prob, int32_t duplicate_factor, uint64_t seed, int32_t bin_size,
                       int64_t *out_totals, void *stream);

/* d_ids: the dense ids lddl_tokenize wrote (and the pack call read).
 * Write the rows of `pack` in output order (partition-major,
 * bin-major, shuffled order within a bin = the reference's part.{p}.parquet_{b}
 * row order).  Row g: d_out_tokens[d_out_tok_off[g] .. d_out_tok_off[g+1]) =
 * [CLS] A [SEP] B [SEP] (CodeBERT: [CLS] doc [SEP] code [SEP], or
 * [CLS] code [SEP] when the document has no docstring); len0/len1 = len(A),
 * len(B); flags bit0 = is_random_next, bit1 = segment 0 is followed by [SEP];
 * bin = bin id; part = partition.  d_bin_count (optional) receives
 * int64[n_part][nbins] row counts. */
int lddl_materialize(lddl_ctx *ctx, lddl_pack *pack, const uint16_t *d_ids, uint16_t *d_out_tokens, int64_t *d_out_tok_off,
                     uint16_t *d_out_len0, uint16_t *d_out_len1, uint8_t *d_out_flags, uint8_t *d_out_bin,
                     int64_t *d_out_part, int64_t *d_bin_count, void *stream);

/* The rows of `pack` as SPANS of the dense ids, in
 * lddl_materialize's row order, without copying a token: each segment of a
 * row is one contiguous run of lddl_tokenize's d_out_ids (a document's
 * sentences are contiguous there and a segment is a window of consecutive
 * sentences), so row g = [CLS] ids[src0[g], src0[g] + len0[g]) [SEP]
 * ids[src1[g], src1[g] + len1[g]) [SEP] (CodeBERT: the [SEP] after segment 0
 * only when flags bit1) -- the same rows as lddl_materialize (binning.py:63-93,
 * pretrain.py:348-353) for consumers that read the ids through the spans
 * (lddl_render_strings RENDER_SPAN: the parquet writer's string columns).
 * len0/len1/flags/bin/part/bin_count as lddl_materialize; d_out_tok_off
 * (optional, NULL = not written) = the materialised layout's row offsets.
 * The dense ids must stay live while the spans are read. */
int lddl_row_spans(lddl_ctx *ctx, lddl_pack *pack, int64_t *d_out_src0, int64_t *d_out_src1, int64_t *d_out_tok_off,
                   uint16_t *d_out_len0, uint16_t *d_out_len1, uint8_t *d_out_flags, uint8_t *d_out_bin,
                   int64_t *d_out_part, int64_t *d_bin_count, void *stream);

/* After lddl_pack_bert(masking=1) + lddl_materialize: apply the masking to
 * the materialised rows in place (A/B become output_tokens[1:1+len(A)] /
 * [2+len(A):...], pretrain.py:232-233) and write, per row g,
 * d_out_mlm_pos[d_out_mlm_off[g] .. d_out_mlm_off[g+1]) = masked_lm_positions
 * (ascending, row coordinates incl. [CLS]) and d_out_mlm_label[...] =
 * masked_lm_labels as token ids (pretrain.py:225-238, :340-361).  Reads
 * the rows and their partitions (d_out_tokens, d_out_tok_off, d_out_part)
 * of that lddl_materialize call, which must still be live. */
int lddl_masked_lm(lddl_ctx *ctx, lddl_pack *pack, int64_t *d_out_mlm_off, uint16_t *d_out_mlm_pos, uint16_t *d_out_mlm_label,
                   void *stream);

/* After lddl_pack_bert(masking=1) + lddl_row_spans (no rows materialised):
 * the static masking of the rows the spans describe.  Per row g,
 * d_out_mlm_off / _pos / _label exactly as lddl_masked_lm, and
 * d_out_mlm_token[k] = the token the masked row shows at position
 * d_out_mlm_pos[k] (the replacement id, or the label when the 10 % "keep"
 * branch left it, pretrain.py:212-225) -- what lddl_render_masked puts into
 * the A / B strings.  d_ids = the dense ids; d_src0 / d_src1 / d_len0 /
 * d_part = that lddl_row_spans call's outputs. */
int lddl_masked_lm_spans(lddl_ctx *ctx, lddl_pack *pack, const uint16_t *d_ids, const int64_t *d_src0, const int64_t *d_src1,
                         const uint16_t *d_len0, const int64_t *d_part, int64_t *d_out_mlm_off,
                         uint16_t *d_out_mlm_pos, uint16_t *d_out_mlm_label, uint16_t *d_out_mlm_token,
                         void *stream);

/* Render one string column of rows [row0, row0 + n_rows) as Arrow string
 * data: d_out_off[0..n_rows] (int64, d_out_off[0] = 0) and the UTF-8 bytes of
 * ' '.join(vocab[t] for t in segment) per row -- the reference's
 * 'A'/'B' (pretrain.py:348-353), 'masked_lm_labels' (:356-360),
 * 'doc'/'code' (pretrain_codebert.py:425-432) columns, which to_parquet
 * writes as pa.string() (pretrain.py:457-471).  segment: 0 = first segment
 * (A / doc: row tokens [1, 1 + len0)), 1 = second (B / code, after the [SEP];
 * codebert != 0: a [SEP] follows the doc segment only when flags bit1),
 * 2 = the whole row (d_row_off only; masked_lm labels from lddl_masked_lm),
 * 3 = a span (lddl_row_spans): row r = d_tokens[d_row_off[r], d_row_off[r] +
 * d_len0[r]) with d_tokens = the dense ids, d_row_off = src0 or src1, d_len0 =
 * len0 or len1 (d_row_off then has n rows, not n + 1 offsets).
 * Two-phase: *out_nbytes receives the byte count (the stream is synchronised
 * once); with d_out_bytes == NULL that is all (size query), else out_cap
 * must be >= it (LDDL_ECAPACITY) and the bytes are written asynchronously. */
int lddl_render_strings(lddl_ctx *ctx, const uint16_t *d_tokens, const int64_t *d_row_off, const uint16_t *d_len0,
                        const uint16_t *d_len1, const uint8_t *d_flags, int64_t row0, int64_t n_rows,
                        int32_t segment, int32_t codebert, int64_t *d_out_off, uint8_t *d_out_bytes,
                        int64_t out_cap, int64_t *out_nbytes, void *stream);

/* The masked rows' A (segment 0) or B (segment 1) strings from the spans:
 * lddl_render_strings' span rendering (d_src / d_len = src0 / len0 or src1 /
 * len1 of lddl_row_spans over d_ids) where a row position listed in
 * d_mlm_pos[d_mlm_off[r] .. d_mlm_off[r+1]) shows d_mlm_token instead
 * (lddl_masked_lm_spans; A's token k sits at row position 1 + k, B's at
 * len0 + 2 + k): the 'A' / 'B' of pretrain.py:232-233, 348-353 with --masking.
 * Same two-phase size query / capacity rules as lddl_render_strings. */
int lddl_render_masked(lddl_ctx *ctx, const uint16_t *d_ids, const int64_t *d_src, const uint16_t *d_len,
                       const uint16_t *d_len0, int32_t segment, const int64_t *d_mlm_off, const uint16_t *d_mlm_pos,
                       const uint16_t *d_mlm_token, int64_t row0, int64_t n_rows, int64_t *d_out_off,
                       uint8_t *d_out_bytes, int64_t out_cap, int64_t *out_nbytes, void *stream);

/* The 'masked_lm_positions' column (pretrain.py:356-360: serialize_np_array
 * of the row's uint16 positions = np.save bytes, lddl/utils.py:98-102) of
 * rows [row0, row0 + n_rows) as Arrow binary data: row r's k =
 * d_mlm_off[r+1] - d_mlm_off[r] positions d_mlm_pos[d_mlm_off[r] ..] (from
 * lddl_masked_lm[_spans], absolute row numbering) become header k + the k
 * values little-endian, where d_hdr holds the np.save header of a uint16[k]
 * array for every k in [0, kmax], hdr_len bytes each (np.save pads every 1-D
 * header to the same length; even).  A row with more than kmax positions is
 * LDDL_EINVAL.  Same two-phase size query / capacity rules as
 * lddl_render_strings. */
int lddl_render_npy(lddl_ctx *ctx, const int64_t *d_mlm_off, const uint16_t *d_mlm_pos, int64_t row0,
                    int64_t n_rows, const uint16_t *d_hdr, int32_t hdr_len, int32_t kmax, int64_t *d_out_off,
                    uint8_t *d_out_bytes, int64_t out_cap, int64_t *out_nbytes, void *stream);

/* Document index (into the corpus' documents) of every row of `pack`, in lddl_materialize's row order: the row's own document (seg0's; a
 * CodeBERT row without docstring: its code's) -- feeds CodeBERT's 'id'
 * column = document._id (pretrain_codebert.py:425-426). */
int lddl_row_docs(lddl_ctx *ctx, lddl_pack *pack, int64_t *d_out_doc, void *stream);

/* Group n rows by length bin exactly as binning.py:63-93
 * _to_dataframe_binned: row i goes to bin (num_tokens[i] - 1) // bin_size
 * (Python floor division), capped at nbins - 1; a negative bin indexes the
 * bins from the end as the reference's seqs[bin_id] does (length 0 -> the
 * last bin), below -nbins is the reference's IndexError (LDDL_EINDEX).
 * d_out_perm[0..n) = the row indices bin-major, ascending within a bin (the
 * row order of the concatenated per-bin frames); d_out_bin_counts[0..nbins)
 * = rows per bin.  1 <= nbins <= 1024, bin_size >= 1.  Synchronises the
 * stream once (the IndexError check). */
int lddl_bin(lddl_ctx *ctx, const int64_t *d_num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
             int64_t *d_out_perm, int64_t *d_out_bin_counts, void *stream);

/* ---- training-time collate -------------------------
 * Replaces lddl/torch/bert.py:69-153 `_to_encoded_inputs` (+ :156-196
 * `_mask_tokens`) for a batch of parquet rows.  Columns arrive as Arrow-style
 * string columns on the device: bytes + int64 offsets[n_rows + 1].
 *
 * lddl_collate_seq_len: the batch's padded length = max over rows of
 * len(A.split()) + len(B.split()) + 3, rounded up to seq_align
 * (bert.py:94-101).  Synchronises the stream (the length shapes the outputs). */
int lddl_collate_seq_len(lddl_ctx *ctx, const uint8_t *d_a, const int64_t *d_a_off, const uint8_t *d_b,
                         const int64_t *d_b_off, int64_t n_rows, int32_t seq_align, int64_t *out_seq_len,
                         void *stream);

/* Fill the [n_rows, seq_len] int64 outputs (bert.py:102-152): input_ids
 * ([CLS] A [SEP] B [SEP], tokens -> ids via the vocab, [UNK] for a miss, 0
 * padding), token_type_ids, attention_mask, next_sentence_labels[n_rows] and
 * d_labels by mode:
 *   0  special_tokens_mask (bert.py:117-122; dynamic masking left to
 *      lddl_mask_tokens);
 *   1  static masking labels: ignore_index except labels[positions] =
 *      ids(labels.split()), positions = the row's np.save uint16 bytes
 *      (d_pos / d_pos_off, d_lab / d_lab_off required);
 *   2  dynamic masking fused: mode 0 then lddl_mask_tokens with the same seed
 *      and counter (identical result).
 * Errors: LDDL_ECAPACITY (a row longer than seq_len, seq_len > 2048),
 * LDDL_EINDEX (a masked position >= seq_len: bert.py:113's IndexError),
 * LDDL_EFORMAT (positions not np.save bytes, or count != label count). */
int lddl_collate_bert(lddl_ctx *ctx, const uint8_t *d_a, const int64_t *d_a_off, const uint8_t *d_b,
                      const int64_t *d_b_off, const uint8_t *d_is_random_next, const uint8_t *d_pos,
                      const int64_t *d_pos_off, const uint8_t *d_lab, const int64_t *d_lab_off, int64_t n_rows,
                      int64_t seq_len, int32_t mode, int64_t ignore_index, double mlm_probability, uint64_t seed,
                      uint64_t counter, int64_t *d_input_ids, int64_t *d_token_type_ids,
                      int64_t *d_attention_mask, int64_t *d_labels, int64_t *d_next_sentence_labels,
                      void *stream);

/* Dynamic MLM masking in place (bert.py:156-196 `_mask_tokens`): a column
 * with special_tokens_mask == 0 is selected with probability
 * mlm_probability; selected -> [MASK] (p 0.8), else a uniform id in
 * [0, vocab size) (p 0.5), else kept; labels = the original id where
 * selected, ignore_index elsewhere.  Draws are a counter-based hash of
 * (seed, counter, row, column): the reference's distribution, not torch's
 * CPU generator stream. */
int lddl_mask_tokens(lddl_ctx *ctx, int64_t *d_inputs, const int64_t *d_special_tokens_mask, int64_t *d_labels,
                     int64_t n_rows, int64_t seq_len, double mlm_probability, int64_t ignore_index, uint64_t seed,
                     uint64_t counter, void *stream);

#ifdef __cplusplus
}
#endif
#endif
