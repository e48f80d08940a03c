// LDS fragment geometry of gemm_s3.h (fp32 operands split into bf16 planes
// while staging): the 32x32x16 fragment of lane l is 8 consecutive k of row
// l&31 (one ds_read_b128), and 40-bf16 (80 B) LDS rows spread every 16-lane
// ds_read_b128 group over all 16 slots of a bank row.  gemm_s3 serves the
// shapes the twin GEMM (gemm_h.h) declines and the DDPG_GEMM_H=0 switch; the
// bf16 configuration otherwise runs gemm_h16_kernel.
#pragma once
#include "gemm_common.h"

namespace ddpg {

constexpr int H_BM = 128, H_BN = 128;
constexpr int H_ROW = 40;  // bf16 per LDS row (32 k + 8 pad)

}  // namespace ddpg
