// Row -> string column rendering and row -> document lookup (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pack.h"

namespace lddl {

// RENDER_SPAN: row r = tokens[row_off[r], row_off[r] + len0[r]) (lddl_row_spans' src / len over the dense ids)
enum : int32_t { RENDER_SEG0 = 0, RENDER_SEG1 = 1, RENDER_ROW = 2, RENDER_SPAN = 3 };

struct RenderParams {
  const uint16_t* tokens;   // rows (lddl_materialize), masked_lm labels, or the dense ids (RENDER_SPAN)
  const int64_t* row_off;   // [rows + 1]; RENDER_SPAN: [rows] segment starts
  const uint16_t* len0;     // RENDER_SEG0/1
  const uint16_t* len1;     // RENDER_SEG1
  const uint8_t* flags;     // RENDER_SEG1 with codebert
  int64_t row0, n_rows;
  int32_t segment, codebert;
  const uint32_t* vinfo;    // [V] pool offset << 8 | byte length
  const uint8_t* vpool;
  int32_t* lens;            // [n_rows] scratch
  const int64_t* out_off;   // [n_rows + 1] (render_bytes)
  uint8_t* out;
  // RENDER_SPAN with static masking (lddl_render_masked): row r's positions
  // mpos[moff[r] .. moff[r+1]) (row coordinates, ascending) show mtok; the
  // span's token k sits at row position 1 + k (A: mseg 0) or len0m[r] + 2 + k (B: mseg 1)
  const int64_t* moff;
  const uint16_t* mpos;
  const uint16_t* mtok;
  const uint16_t* len0m;
  int32_t mseg;
};

struct RowDocParams {
  const PairRec* pairs;
  const int32_t* binned;
  const int64_t* pair_base;
  const int64_t* fs_base;
  const int64_t* sent_off;
  const int64_t* doc_sent_off;
  const int64_t* part_doc_off;
  int64_t n_part, n_rows;
  int32_t dup;
  int64_t* out_doc;
};

// masked_lm_positions as np.save bytes (lddl_render_npy): row r = header of
// its count k (hdr[k], hdr_u16 u16 units, the same length for every k) +
// its k positions as little-endian uint16
struct NpyParams {
  const int64_t* moff;      // [rows + 1] (absolute row numbering)
  const uint16_t* mpos;
  int64_t row0, n_rows;
  const uint16_t* hdr;      // [(kmax + 1) * hdr_u16]
  int32_t hdr_u16, kmax;
  int32_t* lens;            // [n_rows] scratch
  int32_t* err;             // set when a row has more than kmax positions
  const int64_t* out_off;   // [n_rows + 1]
  uint8_t* out;
};

hipError_t launch_render_len(const RenderParams& R, int n_cu, hipStream_t s);
hipError_t launch_npy_len(const NpyParams& N, int n_cu, hipStream_t s);
hipError_t launch_npy_bytes(const NpyParams& N, int n_cu, hipStream_t s);
hipError_t launch_render_bytes(const RenderParams& R, int n_cu, hipStream_t s);
hipError_t launch_row_docs(const RowDocParams& D, int n_cu, hipStream_t s);

}  // namespace lddl
