// Row -> string column rendering and row -> document lookup (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pack.h"

namespace lddl {

enum : int32_t { RENDER_SEG0 = 0, RENDER_SEG1 = 1, RENDER_ROW = 2 };

struct RenderParams {
  const uint16_t* tokens;   // rows (lddl_materialize) or masked_lm labels
  const int64_t* row_off;   // [rows + 1]
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

hipError_t launch_render_len(const RenderParams& R, int n_cu, hipStream_t s);
hipError_t launch_render_bytes(const RenderParams& R, int n_cu, hipStream_t s);
hipError_t launch_row_docs(const RowDocParams& D, int n_cu, hipStream_t s);

}  // namespace lddl
