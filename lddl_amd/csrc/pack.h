// Pair packing + binning + materialisation (device side of lddl_pack_* /
// lddl_materialize).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lddl {

// One packed instance.  BERT: seg0 = A, seg1 = B; CodeBERT: seg0 = doc,
// seg1 = code.  A segment is the concatenation of n filtered sentences
// starting at filtered-sentence slot fs, cut to the token window [lo, hi).
struct PairRec {
  int64_t fs0, fs1;
  uint16_t lo0, hi0, lo1, hi1;
  uint16_t n0, n1;
  uint16_t flags;       // bit0 is_random_next; bit1 seg0 present (CodeBERT [SEP] after doc)
  uint16_t num_tokens;
};
static_assert(sizeof(PairRec) == 32, "PairRec is 32 B");

enum : int32_t { PACK_OK = 0, PACK_EASSERT = 1, PACK_EINDEX = 2, PACK_ELIMIT = 3 };

struct PackParams {
  // tokenizer output + corpus structure
  const int32_t* ntok;          // [n_sent]
  const int64_t* sent_off;      // [n_sent+1] byte offsets (token base = sent_off[s]-sent_off[0])
  const int64_t* doc_sent_off;  // [n_doc+1]
  const int64_t* part_doc_off;  // [n_part+1]
  const int32_t* doc_nseg_doc;  // [n_doc] CodeBERT: # leading docstring segments (else null)
  int64_t n_part;
  // configuration (reference flag names)
  int32_t max_seq;              // --target-seq-length
  int32_t dup;                  // --duplicate-factor
  double short_seq_prob;        // --short-seq-prob
  uint64_t seed;                // partition p uses random.seed(seed + p)
  const uint32_t* mt_states;    // [n_part][MT_N]: those seeded states (launch_mt_seed_states)
  int32_t bin_size;             // --bin-size (or max_seq when unbinned)
  int32_t nbins;                // max_seq // bin_size (1 when unbinned)
  // scratch, indexed like the corpus (sentence / doc / partition slots)
  uint16_t* fs_ntok;            // [n_sent] token count per filtered slot (<= max_tok; u16: half the L2 footprint of the random-next reads)
  int64_t* fs_base;             // [n_sent] byte offset (sent_off - base) per filtered slot (row_docs)
  int64_t* fs_dense;            // [n_sent] dense id offset (tokoff) per filtered slot
  const int64_t* tokoff;        // [n_sent+1] exclusive scan of ntok: sentence s's ids in the dense array
  int64_t* fd_first;            // [n_doc]
  int32_t* fd_n;                // [n_doc]
  int32_t* fd_nd;               // [n_doc] CodeBERT docstring segment count
  PairRec* pairs;               // [dup * n_sent]
  int32_t* order;               // [dup * n_sent]
  int32_t* binned;              // [dup * n_sent]
  int64_t* tok_local;           // [dup * n_sent]
  int64_t* part_npairs;         // [n_part]
  int64_t* part_ntok;           // [n_part]
  int64_t* bin_count;           // [n_part * nbins]
  int64_t* bin_cursor;          // [n_part * nbins] scratch (nbins > 16)
  int32_t* part_err;            // [n_part]
  int32_t* kept;                // [n_sent + n_part] wave packer scratch
  int32_t cap_lens, cap_docs, cap_pairs;  // wave packer: dynamic LDS capacities (per partition)
  uint64_t* dbg;                // wave packer phase cycles (LDDL_PACK_DEBUG=1), else null
  // static masking (create_masked_lm_predictions, pretrain.py:182-238)
  int32_t masking;
  double mlm_ratio;             // --masked-lm-ratio
  uint32_t n_vocab;             // len(vocab_words); vocab_words[i] = token id i
  uint32_t cls_id, sep_id, mask_id;
  const uint8_t* sent_spec;     // [n_sent] sentence holds a [CLS]/[SEP] token
  const uint16_t* ids;          // tokenizer output (dense: sentence s at tokoff[s])
  uint8_t* fs_spec;             // [n_sent] sent_spec per filtered slot
  int64_t* mref;                // [dup*n_sent] per record: arena offset | #masked << 48
  int64_t* mloc;                // [dup*n_sent] per binned position: masked entries before it
  int64_t* part_nmask;          // [n_part]
  uint32_t* marena;             // masked entries: position | (new id or 0xFFFF = keep) << 16
  uint64_t mcap;                // arena capacity (entries)
  unsigned long long* mcounter; // arena bump allocator (entries handed out)
  uint16_t* mcand;              // [n_part * MLM_MAX_SEQ] masking: candidate list scratch per partition
};

constexpr int MLM_CHUNK = 1024;     // arena entries grabbed per allocation
constexpr int MLM_MAX_SEQ = 1024;   // masking: target_seq_length limit (LDS lists)
constexpr uint32_t MLM_KEEP = 0xFFFFu;

struct MlmParams {
  const int64_t* doc_sent_off;
  const int64_t* part_doc_off;
  const int64_t* pair_base;
  const int32_t* binned;
  const int64_t* mref;
  const int64_t* mloc;
  const int64_t* mask_base;     // [n_part+1] exclusive scan of part_nmask
  const uint32_t* marena;
  int64_t n_part;
  int32_t dup;
  uint16_t* tokens;             // rows written by lddl_materialize (masked in place)
  const int64_t* tok_off;
  const int64_t* row_part;      // [n_pairs] partition of each row (materialize's out_part)
  int64_t* out_off;             // [n_pairs+1]
  uint16_t* out_pos;            // [n_masked]
  uint16_t* out_label;          // [n_masked]
  // span mode (tokens == nullptr): the rows as lddl_row_spans described them
  const uint16_t* ids;          // the dense ids
  const int64_t* src0;
  const int64_t* src1;
  const uint16_t* len0;
  uint16_t* out_token;          // [n_masked] the token the masked row holds at out_pos
};

struct MatParams {
  const uint16_t* dense;        // the tokenizer's dense ids (sentence s at tokoff[s])
  const int64_t* fs_dense;      // dense offset per filtered slot
  const int64_t* sent_off;
  const int64_t* doc_sent_off;
  const int64_t* part_doc_off;
  const int64_t* fs_base;
  const uint16_t* fs_ntok;
  const PairRec* pairs;
  const int32_t* binned;
  const int64_t* tok_local;
  const int64_t* part_npairs;
  const int64_t* pair_base;     // [n_part+1] exclusive scan of part_npairs
  const int64_t* tok_base;      // [n_part+1] exclusive scan of part_ntok
  const int32_t* chunk_part;    // row spans: partition of row 64c, per 64-row chunk c (chunk_parts_kernel)
  const int64_t* part_pb;       // row spans: dup * first sentence of partition p (its pair arrays' base)
  int64_t n_part;
  int32_t dup;
  int32_t bin_size, nbins;
  uint32_t cls_id, sep_id;
  int32_t codebert;
  // outputs, global final order (partition-major, bin-major, shuffled)
  uint16_t* out_tokens;         // [total tokens]  [CLS] A [SEP] B [SEP]
  int64_t* out_tok_off;         // [n_pairs + 1]
  uint16_t* out_len0;           // [n_pairs] len(A) / len(doc)
  uint16_t* out_len1;           // [n_pairs] len(B) / len(code)
  uint8_t* out_flags;           // [n_pairs] bit0 is_random_next, bit1 seg0 present
  uint8_t* out_bin;             // [n_pairs]
  int64_t* out_part;            // [n_pairs] partition id (for ids / file names)
  int64_t* out_src0;            // lddl_row_spans: [n_pairs] dense-id offset of segment A / doc
  int64_t* out_src1;            //                 [n_pairs] of segment B / code
};

// random.seed(seed + p) for p < n_part: states[p * MT_N ..] = the MT19937 state
// (states holds ceil(n_part / 64) * 64 rows)
hipError_t launch_mt_seed_states(uint64_t seed, int64_t n_part, uint32_t* states, hipStream_t s);
hipError_t launch_pack_bert_wave(const PackParams& P, hipStream_t s);
size_t pack_dyn_bytes(int cap_lens, int cap_docs, int cap_pairs, bool mask);
hipError_t launch_pack_codebert_wave(const PackParams& P, hipStream_t s);
hipError_t launch_scan_parts(const int64_t* a, const int64_t* b, int64_t n, int64_t* sa, int64_t* sb,
                             const int32_t* err, int32_t* err_any, hipStream_t s);
// algo 1: wave per partition (u16 copies); otherwise wave per 64 pairs with
// 16-B stores (needs out_tokens 16-B aligned and dense padded by 16 u16)
hipError_t launch_materialize(const MatParams& M, int64_t total_pairs, int64_t n_dense, int algo, hipStream_t s);
// row g's segments as offsets into the dense ids (no token copy); out_tok_off optional
hipError_t launch_row_spans(const MatParams& M, int64_t total_pairs, hipStream_t s);
hipError_t launch_chunk_parts(const int64_t* pair_base, const int64_t* doc_sent_off, const int64_t* part_doc_off,
                              int32_t dup, int64_t n_part, int32_t* chunk_part, int64_t* part_pb, hipStream_t s);
// tokoff[0..n] = exclusive scan of ntok[0..n) (int64); blocksums: scratch of
// scan_blocks(n) + 1 entries
__host__ __device__ int64_t scan_blocks(int64_t n);
hipError_t launch_scan_ntok(const int32_t* ntok, int64_t n, int64_t* tokoff, int64_t* blocksums, hipStream_t s);
// the same over [*d_lo, *d_hi) (device values, at most max_items), continuing
// from tokoff[*d_lo]; blocksums: scan_blocks(max_items) + 1
hipError_t launch_scan_ntok_range(const int32_t* ntok, const int64_t* d_lo, const int64_t* d_hi, int64_t max_items,
                                  int64_t* tokoff, int64_t* blocksums, hipStream_t s);
// lddl_bin (bin.hip): stable grouping of rows by length bin.  hist:
// bin_chunks(n) * nbins int32, base: that + 1 int64, scan_bsum:
// scan_blocks(that) + 1 int64; err[0] = 1 when a bin is below -nbins
int64_t bin_chunks(int64_t n);
hipError_t launch_bin(const int64_t* num_tokens, int64_t n, int32_t bin_size, int32_t nbins, int32_t* hist,
                      int64_t* base, int64_t* scan_bsum, int64_t* perm, int64_t* bin_counts, int32_t* err,
                      hipStream_t s);
hipError_t launch_sent_special(const uint16_t* ids, const int64_t* tok_off, const int32_t* ntok, int64_t n_sent,
                               uint32_t cls, uint32_t sep, uint8_t* out, hipStream_t s);
hipError_t launch_masked_lm(const MlmParams& M, int64_t n_rows, hipStream_t s);

}  // namespace lddl
