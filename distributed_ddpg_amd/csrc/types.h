// Argument structs and configuration constants shared by the kernels and the
// host code (the C-ABI translation units include this without the kernels):
// the fused GEMM epilogue, the thin-K layer parts, the small-batch path's
// saved-tensor layout and weight-gradient tables.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddpg {

// ---------------------------------------------------------------- GEMMs (gemm_common.h)
enum { L_RK = 0, L_KR = 1 };

// in-launch K split (ksplit_combine, gemm_common.h): at most KC_MAXS splits
// per tile (DDPG_KCOMB_SPLITS=2 / 3 lowers the cap; 8 splits measured slower
// at the per-rank B = 512 shapes, profiles/r4/per_rank_split8.txt)
constexpr int KC_MAXS = 4;
constexpr int GBK = 32, GNT = 256;
constexpr int PROJ_MAX = 32;

template <int BM, int BN>
struct TileCfg {
  static constexpr int STAGE = 2 * GBK * (BM + 1) + 2 * GBK * (BN + 1);
  static constexpr int VS_LD = BN + 4;
  static constexpr int EPI = (BM / 2) * VS_LD + BN * PROJ_MAX + 2 * GNT;  // red: up to 512 threads
  static constexpr int SMEM = STAGE > EPI ? STAGE : EPI;
};

struct GemmEpi {
  float* out;
  long long out_split_stride;
  int ldo;
  int act;   // 0 none, 1 elu
  int post;  // 0 none, 1 mul elu'(aux), 2 pw[n] * elu'(v)
  int ldaux;
  const float* bias;
  const float* aux;
  const float* pw;
  float* colsum;  // [split * mtiles + mtile][ld_colsum]
  int ld_colsum;
  int proj_n, proj_sn, proj_sa;
  const float* proj;  // Wp[n][a] = proj[n * proj_sn + a * proj_sa]
  float* proj_out;    // [ntile][M][proj_n]
  // bf16 twin of out (same element offsets, ld = ldo): h_planes = 1 stores
  // bf16(v); 3 stores the exact h/m/l split of v, planes h_plane_stride apart.
  // Read by the bf16-operand GEMM (gemm_h.h).  Needs N, ldo % 4 == 0.
  __bf16* outh;
  long long h_plane_stride;
  int h_planes;
  // post 1 with auxh (and aux == nullptr): the EluGrad operand is read from
  // its three exact bf16 planes ((h + m) + l == the fp32 value), offsets and
  // ld as aux, planes auxh_ps apart -- for activations whose fp32 copy is not
  // written (fp32 contexts whose other readers all take the twin)
  const __bf16* auxh;
  long long auxh_ps;
  // fp32 `out` stored only for columns n >= out_col0 (the twin for all): an
  // output whose leading columns have twin readers only
  int out_col0;
  // Narrow weight gradient of the NEXT layer down, from this dX tile (the
  // input layers' dW1 = s^T dz1, dWs = s^T dcat_s, dWa = a^T dcat_a with a
  // <= 64-wide narrow side): the tile's final values v (rows m0 .. m0 + BM,
  // columns n0 .. n0 + BN) times the narrow operand's rows, one partial per
  // row tile and row group into nw_out[set] + (by * nw_rg + g) * nw_slab
  // ([nw_k][nw_ld] each; grad_reduce sums the slabs).  Set 1 (if any) takes the
  // columns n >= nw_col1 (dcat's action half).  One-pass epilogues only.
  const float* nw_x[2];  // narrow operand [M][nw_ldx], 16-B rows
  int nw_ldx[2], nw_k[2], nw_ld[2], nw_rg[2];
  float* nw_out[2];
  long long nw_slab[2];
  int nw_col1;
};

struct GemmArgs {
  const float* A;
  const float* B;
  int M, N, K, lda, ldb;
  int kps;  // k extent per split (multiple of GBK)
  int xcd;  // 1: XCD-aware tile order (xcd_tile)
  GemmEpi e;
};

// ---------------------------------------------------------------- thin-K layers (thin_k.h)
constexpr int TK_MAXK = 64;
#ifndef TK_COLS_CFG
#define TK_COLS_CFG 128
#endif
constexpr int TK_ROWS = 64, TK_COLS = TK_COLS_CFG, TK_NT = 256;
static_assert(TK_COLS == 64 || TK_COLS == 128, "thin_k column block");
constexpr int TK_TPW = TK_COLS / 64;       // 32x32 tiles per wave (4 waves: 2 x 2)
constexpr int TK_KQS = TK_NT / TK_COLS;    // k-quad stride of the W panel loads
constexpr int TK_WJ = 16 / TK_KQS;         // W panel float4 loads per thread
constexpr int TK_OCT = TK_COLS / 8;        // column octets of the epilogue
constexpr int TK_RG = TK_NT / TK_OCT;      // epilogue row groups
constexpr int TK_KALIGN = 8;

struct TkPart {
  const float* X;   // [M][ldx], 16-byte aligned, ldx % 4 == 0
  int ldx, K;       // K % 8 == 0
  const float* W;   // w_nk ? W[n][k] (ldw) : W[k][n] (ldw); 16-byte aligned, ldw % 4 == 0
  int ldw, w_nk;
  int N;              // N % 4 == 0
  const float* bias;  // [N] or null
  int act;            // 1: elu
  const float* aux;   // v *= EluGrad factor of aux[m][n] (ldaux), or null
  int ldaux;
  float* out;         // out[m * ldo + n]
  int ldo;
  __bf16* outh;       // bf16 twin of out (same offsets; hnp planes, hps apart), or null
  long long hps;
  int hnp;
  float* colsum;      // [row block][ld_colsum] partial column sums of v, or null
  int ld_colsum;
  // backward form only: the weight gradient aux^T X of the layer whose output
  // gradient X is (dW3 = h2^T dz3 beside dz2), one fp32 partial per row tile:
  // dw[rt * dw_slab + n * dw_k + a], a < dw_k <= K <= 32; null: not fused
  float* dw;
  int dw_k;
  long long dw_slab;
};

constexpr int TK_MAXP = 5;  // parts per launch (blockIdx.z)

struct TkArgs {
  TkPart p[TK_MAXP];
  int M;
  int mt;   // row tiles (ceil(M / TK_ROWS))
  int rpb;  // row tiles per block (blockIdx.y owns [rpb * y, rpb * y + rpb))
};

// LDS: the W image (3 planes, resident for the whole block), then one region
// shared by the X image (3 planes) of the current row tile and, after its
// MFMAs, the raw output tile [64 rows][TK_COLS] (16-B chunks XOR-swizzled by
// row: tk_oidx), then the column-sum scratch of the epilogue.
constexpr int TK_XIMG = TK_ROWS * 128;  // bytes per X plane
constexpr int TK_WIMG = TK_COLS * 128;  // bytes per W plane
constexpr int TK_OUT_BYTES = TK_ROWS * TK_COLS * 4;
constexpr int TK_XREG = 3 * TK_XIMG > TK_OUT_BYTES ? 3 * TK_XIMG : TK_OUT_BYTES;
constexpr int TK_LDS = 3 * TK_WIMG + TK_XREG;
static_assert(TK_LDS <= 80 * 1024, "two blocks per CU");
static_assert(TK_RG * TK_COLS * 4 <= TK_XREG, "column-sum scratch aliases the output tile");
static_assert((32 * TK_COLS + 32 * 32) * 4 <= TK_XREG, "fused dW staging aliases the output tile");

// ---------------------------------------------------------------- small-batch path (small_batch.h)
// Saved per-row tensors that the weight gradients read, feature-major
// ([feature][Bp], Bp = Bmax rounded up to 4): a workgroup stores its 4 rows of
// a feature as one float4 and the gradient kernel reads a feature's batch
// column as contiguous float4s.
struct SbSave {
  int Bp;
  float *xs, *xa;          // [S], [A]      inputs (scaled)
  float *cat, *dcat;       // [2 CH1]       critic concat, its gradient
  float *h, *dhp;          // [CH2],[CH2]   critic hidden, its pre-act grad / dQ (below)
  float *q, *y;            // [1], [1]      online Q, TD target (ddpg.py:92-97)
  float *h1, *h2;          // [AH1], [AH2]  actor hidden
  float *dz1, *dz2, *dz3;  // [AH1], [AH2], [A]
  float* o;                // [A]           actor output tanh(.) (phase 1 -> phase 3)
};

// One network's weight-gradient table: tensor i occupies param offsets
// [off, off + K*N) (row-major [K][N]); its gradient is
//   g[k][n] = sum_b X[k][b] dY[n][b]   (feature-major saves; X == nullptr: bias, X = 1)
// over the B saved rows, computed by tiles of TK x TN elements (TK*TN = SB_GT)
// starting at block tile0.  sdq: the saved dY is the critic's output
// gradient per unit dQ, and dY[n][b] = dQ[b] * saved[n][b] (dY == nullptr:
// dQ itself), dQ formed in the kernel from the saved q and TD target.
struct SbGradT {
  long long off;
  int K, N;
  const float* X;
  int ldx;
  const float* dY;
  int ldy;
  int TN, TK, tile0;
  int sdq;
};
constexpr int SB_MAXT = 10;  // tensors per network + the sentinel
struct SbGradTab {
  SbGradT t[SB_MAXT];
  int n;
  int shadow;  // index of the tensor whose transpose is kept (Wh / W2), -1 none
  float* sh;
};

// twin-GEMM launch arguments (gemm_h.h, gemm_h3.h)
struct GemmHArgs {
  const __bf16* A;
  const __bf16* B;
  long long pa, pb;  // elements between planes (NP = 3)
  int M, N, K, lda, ldb;
  int kps;  // k extent per split (multiple of BK)
  int xcd;
  GemmEpi e;
  // in-launch K split (ksplit_combine, gemm_h3_kernel / gemm_h16i_kernel):
  // partials [tile][split] and one ticket per output tile; null: the splits
  // are separate slabs (weight gradients) or there is one split
  float* kpart = nullptr;
  unsigned* kticket = nullptr;
#ifdef DDPG_KC_STAMPS
  unsigned long long* stamps = nullptr;  // tools/kc_bench.hip only: per-block phase clocks
#endif
};

// independent GEMMs of one grid shape launched together (gemm_h16i_pack_kernel)
constexpr int GH_MAXP = 4;
struct GemmHPack {
  GemmHArgs p[GH_MAXP];
};

}  // namespace ddpg
