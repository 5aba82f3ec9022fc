// Training-time collate of parquet rows into BERT model inputs (device side of
// lddl_collate_seq_len / lddl_collate_bert / lddl_mask_tokens).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lddl {

enum : int32_t { COLLATE_SPECIAL_MASK = 0, COLLATE_STATIC = 1, COLLATE_DYNAMIC = 2 };

// Whole-token vocab table for convert_tokens_to_ids: open addressing over
// slots {hash, id}; the key bytes are verified against the render pool
// (vinfo[id] = offset << 8 | length, the full entry text incl. "##").
struct CollateVocab {
  const uint2* slots;
  uint32_t mask;
  const uint32_t* vinfo;
  const uint8_t* vpool;
  int32_t unk, cls, sep, mask_id;
  int32_t n_random;  // len(tokenizer): randint bound of the 10 % random words
};

struct CollateParams {
  CollateVocab V;
  const uint8_t* a;
  const int64_t* a_off;  // [n_rows + 1]
  const uint8_t* b;
  const int64_t* b_off;
  const uint8_t* is_random_next;  // [n_rows] (bool bytes)
  const uint8_t* pos;             // static masking: np.save bytes per row
  const int64_t* pos_off;
  const uint8_t* lab;             // static masking: space-joined label tokens
  const int64_t* lab_off;
  int64_t n_rows;
  int32_t seq_len;   // output columns (aligned)
  int32_t mode;      // COLLATE_*
  int64_t ignore_index;
  double mlm_probability;
  uint64_t seed, counter;
  int64_t* input_ids;        // [n_rows, seq_len]
  int64_t* token_type_ids;
  int64_t* attention_mask;
  int64_t* labels;           // labels, or special_tokens_mask (COLLATE_SPECIAL_MASK)
  int64_t* next_sentence_labels;  // [n_rows]
  int32_t* max_len;          // [1] max over rows of len(A) + len(B) + 3 (seq-len pass)
  uint32_t* err;             // [1] first error code (0 = none) | row << 4
};

struct MaskParams {
  int64_t* inputs;            // [n_rows, seq_len], masked in place
  const int64_t* special;     // [n_rows, seq_len] special_tokens_mask
  int64_t* labels;            // [n_rows, seq_len]
  int64_t n_rows;
  int32_t seq_len, mask_id, n_random;
  int64_t ignore_index;
  double mlm_probability;
  uint64_t seed, counter;
};

// error codes in CollateParams::err (low 4 bits)
enum : uint32_t { CERR_LONG = 1, CERR_POS_RANGE = 2, CERR_NPY = 3, CERR_NLAB = 4 };

constexpr int COLLATE_MAX_LEN = 2048;  // per-row LDS buffer (columns)

uint32_t collate_hash_host(const uint8_t* p, int n);
hipError_t launch_collate_len(const CollateParams& P, int n_cu, hipStream_t s);
hipError_t launch_collate_fill(const CollateParams& P, int n_cu, hipStream_t s);
hipError_t launch_mask_tokens(const MaskParams& M, int n_cu, hipStream_t s);

}  // namespace lddl
