// GEMM-shaped launches of the learner step: the plan (tile, split-K, the
// small-M in-launch K split, XCD tile order, twin-operand eligibility) and the
// launches of the fp32 / three-plane / bf16 GEMM kernels, the thin-K layers
// and the skinny weight gradients.  DESIGN.md §4.
#include "ctx.h"
#include "gemm_f32.h"
#include "gemm_bf16.h"
#include "gemm_s3.h"
#include "gemm_h.h"
#include "gemm_h256.h"
#include "gemm_h3m.h"
#include "gemm_hw.h"
#include "thin_k.h"
#include "skinny.h"

// Block-count target for tile selection (env DDPG_GEMM_MIN_BLOCKS overrides).
static int g_min_blocks = 1024;

static const int kTiles[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};

// Largest tile (no more than one 64-row/col of padding) whose grid reaches
// the block target; otherwise the one with the most blocks.
static void pick_tile(int M, int N, int min_blocks, int* bm, int* bn) {
  int best = -1, best_blocks = -1;
  for (int t = 0; t < 4; ++t) {
    const int tm = kTiles[t][0], tn = kTiles[t][1];
    if (tm > 64 && M <= 64) continue;
    if (tn > 64 && N <= 64) continue;
    const int blocks = ceil_div(M, tm) * ceil_div(N, tn);
    if (blocks >= min_blocks) {
      *bm = tm;
      *bn = tn;
      return;
    }
    if (blocks > best_blocks) {
      best_blocks = blocks;
      best = t;
    }
  }
  *bm = kTiles[best][0];
  *bn = kTiles[best][1];
}

// Plan for a plain (splits = 1) GEMM or a split-K weight-gradient GEMM
// (splits = 0: auto, ~512 blocks, >= 128 k per split, <= cap).
GemmPlan make_plan(int M, int N, int K, int splits, int cap, bool big) {
  GemmPlan p;
  if (big) {  // bf16 kernel: fixed 128 x 128 tile
    p.bm = p.bn = 128;
    if (splits != 1) {
      const int tiles = ceil_div(M, 128) * ceil_div(N, 128);
      splits = std::max(1, 512 / tiles);
      splits = std::min(splits, std::max(1, K / 128));
      splits = std::min(splits, cap);
    }
  } else if (splits == 1) {
    pick_tile(M, N, g_min_blocks, &p.bm, &p.bn);
  } else {
    p.bm = M <= 64 ? 64 : 128;
    p.bn = N <= 64 ? 64 : 128;
    const int tiles = ceil_div(M, p.bm) * ceil_div(N, p.bn);
    splits = std::max(1, 512 / tiles);
    splits = std::min(splits, std::max(1, K / 128));
    splits = std::min(splits, cap);
  }
  p.kps = rup(std::max(1, ceil_div(K, splits)), GBK);
  p.splits = std::max(1, ceil_div(K, p.kps));
  return p;
}

// Twin of an activation buffer element (nullptr unless the buffer is twinned)
Twin act_twin(const ddpg_ctx* c, const float* q) {
  Twin t;
  if (!c->hnp || !q) return t;
  for (const auto& b : c->twinned)
    if (q >= b.first && q < b.first + b.second) {
      t.p = c->atw + (q - c->dact);
      t.ps = (long long)c->act_n;
      return t;
    }
  return t;
}

// Twin of a GEMM operand: a parameter (theta / target, while the parameter
// twins are current) or a twinned activation buffer
Twin operand_twin(const ddpg_ctx* c, const float* q) {
  Twin t;
  if (!c->hnp || !q) return t;
  const size_t PT = c->L.total;
  if (c->wtw_ok) {
    if (q >= c->theta && q < c->theta + PT) {
      t.p = c->wtw + (q - c->theta);
      t.ps = (long long)PT;
      return t;
    }
    if (q >= c->target && q < c->target + PT) {
      t.p = c->wtw + (size_t)c->hnp * PT + (q - c->target);
      t.ps = (long long)PT;
      return t;
    }
  }
  return act_twin(c, q);
}

// Row buffers whose columns past the logical width are always zero (their
// writers touch only the first S / A columns): a contraction over them may run
// K-padded to its kernel's k step, the padded products being exact zeros.
static bool zero_padded(const ddpg_ctx* c, const float* q) {
  return q == c->s || q == c->s2 || q == c->a || q == c->ta2 || q == c->mu || q == c->dz3;
}

template <int AL, int BL, int VA, int VB>
static void gemm_dispatch(const GemmPlan& p, dim3 grid, hipStream_t st, const GemmArgs& g) {
  if (p.bm == 128 && p.bn == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 128, 128>), grid, dim3(GNT), 0, st, g);
  else if (p.bm == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 128, 64>), grid, dim3(GNT), 0, st, g);
  else if (p.bn == 128)
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 64, 128>), grid, dim3(GNT), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, VA, VB, 64, 64>), grid, dim3(GNT), 0, st, g);
}

// XCD tile order for an nx x ny grid of BM x BN tiles (xcd_tile): the
// rectangle of tiles per XCD with the fewest operand-panel bytes
// (H row panels of BM rows + W column panels of BN columns), when 8 such
// rectangles tile the grid and it reads fewer bytes than the row-major runs.  env DDPG_XCD_RECT=0
// keeps the runs.
static int xcd_rect(const ddpg_ctx* c, int nx, int ny, int BM, int BN) {
  const int on = c->sw.xcd;
  if (!on || !c->sw.xcd_rect || (nx * ny) % 8) return on;
  const int T = nx * ny / 8;
  int best = -1, best_cost = 0;
  for (int W = 1; W <= nx; ++W) {
    if (nx % W || T % W) continue;
    const int H = T / W;
    if (ny % H || (nx / W) * (ny / H) != 8) continue;
    const int cost = H * BM + W * BN;
    if (best < 0 || cost < best_cost) {
      best = W;
      best_cost = cost;
    }
  }
  // keep the row-major runs unless the rectangle reads strictly fewer bytes
  const int run_cost = T % nx ? -1 : (T / nx) * BM + nx * BN;
  if (best < 0 || (run_cost >= 0 && best_cost >= run_cost)) return on;
  return 16 + best;
}

static bool use_bf16(const ddpg_ctx* c, int M, int N, bool vec);
static bool use_s3(const ddpg_ctx* c, int M, int N, bool vec);

// Whether gemm_launch runs this GEMM on the bf16-twin kernel (both operands
// twinned, shapes in its tiles, K in whole k-tiles -- or K-padded first
// layers: A rows zero past K, B a parameter twin whose rows past K are the
// next tensors' finite values, multiplied by zero); *Kh = the K it runs.
// Producers use it to skip fp32 copies nobody reads.
template <int AL, int BL>
bool gemm_h_ok(const ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M,
                      int N, int K, int splits, int* Kh) {
  if (!(c->sw.gemm_h && c->hnp && M >= 128 && N >= 128 && N % 8 == 0 && lda % 8 == 0 &&
        ldb % 8 == 0 && (AL == L_RK || M % 8 == 0) && (BL == L_RK || N % 8 == 0)))
    return false;
  const int BKh = c->hnp == 1 ? 64 : 32;
  const Twin ta = operand_twin(c, A), tb = operand_twin(c, B);
  int k = K;
  if (K % BKh && AL == L_RK && BL == L_KR && zero_padded(c, A) && rup(K, BKh) <= lda && tb.p &&
      tb.ps == (long long)c->L.total && splits == 1)
    k = rup(K, BKh);
  if (!(k % BKh == 0 && ta.p && tb.p && aligned16(ta.p) && aligned16(tb.p))) return false;
  *Kh = k;
  return true;
}

// gemm_h256_kernel (bf16 configuration, 256 x 256 tiles): splits of a
// weight gradient -- about one block per CU, every split a whole number of
// the kernel's 4-step trips (kps % 128 == 0)
static int h256_splits(int M, int N, int K, int cap) {
  const int tiles = (M / H2_BM) * (N / H2_BN);
  int sp = std::max(1, 256 / tiles);
  sp = std::min(std::min(sp, cap), std::max(1, K / 128));
  while (sp > 1 && (K % sp || (K / sp) % 128)) --sp;
  return sp;
}
// -1: not taken; 0: split-K weight gradient with a plain slab epilogue
// (DDPG_GEMM256=1); 1 / 2: unsplit GEMMs (=2 / =3).  Full tiles only.  Off by
// default: in the C5 step the finer split's extra slab reduction cost more
// than the faster main loop saved (profiles/r3/gemm_h256_ab_c5.txt).
static int h256_mode(const ddpg_ctx* c, int M, int N, int Kh, int splits, const GemmEpi& e) {
  if (!(c->hnp == 1 && c->sw.gemm256 && M % H2_BM == 0 &&
        N % H2_BN == 0 && Kh % 128 == 0))
    return -1;
  const bool plain = !e.bias && e.act == 0 && e.post == 0 && !e.colsum && !e.proj_out && !e.outh;
  return splits != 1 && plain ? 0 : -1;
}

// direct: for a split-K weight gradient, where to write the result when the
// plan ends up with one split (no slab, no reduction; plan.direct = true).
template <int AL, int BL>
GemmPlan gemm_launch(ddpg_ctx* c, const char* name, const float* A, int lda,
                            const float* B, int ldb, int M, int N, int K, const GemmEpi& e,
                            int splits, int cap, float* direct) {
  const int contA = (AL == L_RK) ? K : M;
  const int contB = (BL == L_RK) ? K : N;
  const bool va = (contA % 4 == 0) && (lda % 4 == 0) && aligned16(A);
  const bool vb = (contB % 4 == 0) && (ldb % 4 == 0) && aligned16(B);
  const bool vec = va && vb;
  const bool bf = use_bf16(c, M, N, vec);
  const bool s3 = !bf && use_s3(c, M, N, vec);
  GemmPlan p = make_plan(M, N, K, splits, cap, bf || s3);
  if (M <= 0 || N <= 0) return p;
  {  // the element-wise combinations gemm_epilogue is specialised on
    const bool b = e.bias != nullptr;
    const bool ok = (!b && e.act == 0 && e.post == 0) || (b && e.act == 1 && e.post == 0) ||
                    (b && e.act == 1 && e.post == 2) || (!b && e.act == 0 && e.post == 1) ||
                    (b && e.act == 0 && e.post == 0);
    if (!ok) throw einval("gemm %s: unsupported epilogue (bias %d act %d post %d)", name, b, e.act,
                          e.post);
  }
  // a twinned output gets its bf16 twin written by the epilogue
  GemmEpi ee = e;
  if (!ee.outh && ee.out && !ee.out_split_stride) {
    const Twin to = act_twin(c, ee.out);
    if (to.p) {
      ee.outh = to.p;
      ee.h_plane_stride = to.ps;
      ee.h_planes = c->hnp;
    }
  }
  // the fused narrow weight gradient (nw_*) runs in the epilogues of gemm_h3 /
  // gemm_h3m (fp32) and gemm_h16i (bf16, RK A); the caller checked (step.hip nw_ok)
  const bool nwe = e.nw_out[0] || e.nw_out[1];
  // bf16-twin operands (gemm_h.h): both operands twinned, K in whole k-tiles
  int Kh = 0;
  if (gemm_h_ok<AL, BL>(c, A, lda, B, ldb, M, N, K, splits, &Kh)) {
    if (nwe && !((c->hnp == 3 || (c->hnp == 1 && AL == L_RK)) && c->sw.gemm_h3 &&
                 M % (c->hnp == 1 ? 256 : 128) == 0 && N % 128 == 0 && splits == 1))
      throw einval("gemm %s: fused narrow weight gradient needs gemm_h3 / gemm_h16i full tiles",
                   name);
    const int BKh = c->hnp == 1 ? 64 : 32, BMh = c->hnp == 1 ? 256 : 128;
    const Twin ta = operand_twin(c, A), tb = operand_twin(c, B);
    {
      // as requested (the 256 x 128 plan below rewrites both)
      const int splits_req = splits;  // 1: plain GEMM; otherwise a split-K weight gradient
      const GemmEpi ee_req = ee;
      GemmPlan h;
      h.bm = BMh;
      h.bn = HG_BN;
      if (splits != 1) {  // ~one block per CU (144 KB of LDS each)
        const int tiles = ceil_div(M, BMh) * ceil_div(N, HG_BN);
        splits = std::max(1, 256 / tiles);
        splits = std::min(splits, std::max(1, K / (4 * BKh)));
        splits = std::min(splits, cap);
      }
      h.kps = rup(ceil_div(Kh, std::max(1, splits)), BKh);
      h.splits = ceil_div(Kh, h.kps);
      // bf16 weight gradients (KR x KR) on gemm_hw_kernel (128 x 64 wave
      // tiles, 1.2x gemm_h16_kernel): full 256 x 128 tiles, every split a whole
      // number of its 4-step trips (kps % 128 == 0), the split count at most
      // the one planned above
      // (full tiles only: the partial-M dWs / dW1, 376 x 2048, measured 1.02x
      // isolated and no better in the step, profiles/r6/hw_bench_wgrad_partial.txt)
      bool hw = false;
      if (c->hnp == 1 && AL == L_KR && BL == L_KR && c->sw.gemm_hw && M % 256 == 0 &&
          N % HG_BN == 0) {
        for (int sp = h.splits; sp >= 1 && !hw; --sp)
          if (Kh % sp == 0 && (Kh / sp) % 128 == 0) {
            hw = true;
            h.splits = sp;
            h.kps = Kh / sp;
          }
      }
      if (h.splits == 1 && direct) {
        ee.out = direct;
        ee.out_split_stride = 0;
        h.direct = true;
      }
      GemmHArgs a;
      // small-M plan: a plain GEMM (forward / dX) whose tiles leave most CUs
      // idle -- per-rank batches of a strong-scaling run, e.g. C3 at B = 512
      // has 32 forward tiles for 256 CUs -- splits K over ~256 blocks (>= 3
      // k-tiles each) and combines the splits in-launch before its epilogue
      // (ksplit_combine).  The immediate-offset kernels only.
      const bool kc_kernel = c->sw.gemm_h3 && (c->hnp == 3 || (c->hnp == 1 && AL == L_RK));
      // data-parallel steps: a split weight gradient with a direct target
      // combines its splits in-launch too -- the reduced gradient is then
      // written once, in place, and its all-reduce starts right behind the
      // GEMM (a one-rank step leaves the slabs to the Adam pass that reads them)
      const bool kc_wgrad = splits_req != 1 && direct && c->comm && c->hnp == 3 && c->sw.kc_wgrad;
      if ((splits_req == 1 || (kc_wgrad && (h.splits == 2 || h.splits == 4))) && kc_kernel &&
          c->kc_part) {
        const int tiles = h.nt(N) * h.mt(M);
        const int nkt = Kh / BKh;
        int sk = std::min({ceil_div(256, tiles), nkt / 3, c->sw.kc_splits});
        // a weight gradient keeps the slab plan's K ranges: its partials, and
        // their sum in split order, are then those of the slab reduction
        // (slab_partial: ((s0 + s1) + s2) + s3), bit for bit
        if (kc_wgrad) sk = h.splits;
        while (sk > 2 && (size_t)sk * tiles * BMh * HG_BN > c->kc_part_n) --sk;  // partial buffer
        if (tiles < c->sw.kc_blocks && sk >= 2) {
          const int kps = ceil_div(nkt, sk) * BKh;
          sk = ceil_div(Kh, kps);
          if (sk >= 2 && (size_t)sk * tiles * BMh * HG_BN <= c->kc_part_n && tiles <= kKcTickets) {
            const int slot = c->kc_next++ % c->kc_rot;
            a.kpart = c->kc_part + (size_t)slot * c->kc_part_n;
            a.kticket = c->kc_ticket + (size_t)slot * kKcTickets;
            h.kps = kps;
            h.splits = sk;
            if (kc_wgrad) {
              ee.out = direct;
              ee.out_split_stride = 0;
              h.direct = true;
            }
          }
        }
      }
      a.A = ta.p;
      a.B = tb.p;
      a.pa = ta.ps;
      a.pb = tb.ps;
      a.M = M;
      a.N = N;
      a.K = Kh;
      a.lda = lda;
      a.ldb = ldb;
      a.kps = h.kps;
      a.xcd = xcd_rect(c, h.nt(N), h.mt(M), BMh, HG_BN);
      a.e = ee;
      static const char* lay[2] = {"RK", "KR"};
      // bf16 configuration, opt-in DDPG_GEMM256=1: the split-K weight
      // gradients on whole 256 x 256 tiles (gemm_h256.h, plain slabs, MODE 0)
      const int mode256 =
          h256_mode(c, M, N, Kh, splits_req, ee_req);
      if (mode256 >= 0) {
        GemmPlan q;
        q.bm = q.bn = H2_BM;
        const int sp = h256_splits(M, N, Kh, cap);
        q.kps = Kh / sp;
        q.splits = sp;
        GemmEpi e2 = ee_req;
        if (q.splits == 1 && direct) {
          e2.out = direct;
          e2.out_split_stride = 0;
          q.direct = true;
        }
        a.e = e2;
        a.kps = q.kps;
        a.xcd = xcd_rect(c, q.nt(N), q.mt(M), H2_BM, H2_BN);
        char key[112];
        snprintf(key, sizeof key, "gemm_h256_kernel<%s,%s,MODE=%d>|%s", lay[AL], lay[BL], mode256,
                 name);
        ProfScope ps(c, key, 2.0 * M * N * (double)K,
                     2.0 * ((double)M * K + (double)K * N) + 4.0 * (double)M * N * q.splits);
        const dim3 grid(q.nt(N), q.mt(M), q.splits);
        hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 0>), grid, dim3(H2_NT), 0, c->cur, a);
        HIP_TRY(hipGetLastError());
        return q;
      }
      // bf16 configuration: the 16x16x32-MFMA kernels
      const bool h16 = c->hnp == 1;
      // fp32 contexts on the 16x16x32 form: the forward / dX GEMMs unless K is
      // split in-launch (small-M plan: with 8-16 k-tiles per block the
      // 32x32x16 form is 1-2 % faster, per-rank C3 B = 512, profiles/r5/), and
      // the weight gradients (KR x KR) always -- a data-parallel step's
      // in-launch combine then sums the same per-split partials as the
      // one-rank step's slabs
      const bool m16 = c->hnp == 3 && c->sw.gemm_m16 &&
                       ((AL == L_RK && !a.kpart) || (AL == L_KR && BL == L_KR));
      char key[112];
      // "/kc": the splits are combined in-launch (small-M plan)
      // DDPG_PROF_SHAPES=1: the shape and split count in the key too
      char shp[48] = "";
      if (c->sw.prof_shapes) snprintf(shp, sizeof shp, " %dx%dx%d/%d", M, N, K, h.splits);
      snprintf(key, sizeof key, "%s<%s,%s,NP=%d>|%s%s%s",
               hw ? "gemm_hw_kernel"
               : h16 ? (AL == L_RK && c->sw.gemm_h3 ? "gemm_h16i_kernel" : "gemm_h16_kernel")
                   : (c->hnp == 3 && c->sw.gemm_h3) ? (m16 ? "gemm_h3m_kernel" : "gemm_h3_kernel")
                                                    : "gemm_h_kernel",
               lay[AL], lay[BL], c->hnp, name, a.kpart ? "/kc" : "", shp);
      const dim3 grid(h.nt(N), h.mt(M), h.splits);
      const double fl = 2.0 * M * N * (double)K,
                   by = 2.0 * c->hnp * ((double)M * K + (double)K * N) + 4.0 * (double)M * N * h.splits;
      if constexpr (AL == L_RK && BL == L_KR) {
        // gemm_defer (first_layers_dev, learner_step_dev's forward layers):
        // queue for one pack launch -- the kernels with a pack form only
        // (gemm_h16i, gemm_h3m)
        const bool pk_ok = h16 ? c->sw.gemm_h3 : (c->sw.gemm_h3 && m16);
        if (c->gemm_defer && pk_ok && h.splits == 1 && !a.kpart) {
          DeferredGemm d;
          d.a = a;
          d.grid = grid;
          d.flops = fl;
          d.bytes = by;
          snprintf(d.key, sizeof d.key, "%s", key);
          c->deferred.push_back(d);
          return h;
        }
      }
      ProfScope ps(c, key, fl, by);
      if (hw) {
        if constexpr (AL == L_KR && BL == L_KR)
          hipLaunchKernelGGL((gemm_hw_kernel<AL, BL, HG_BN, 4>), grid, dim3(2 * HG_BN), 0, c->cur, a);
      } else if (h16 && AL == L_RK && c->sw.gemm_h3) {
        // immediate-offset addressing (gemm_h3.h), RK A operands
        if constexpr (AL == L_RK)
          hipLaunchKernelGGL((gemm_h16i_kernel<AL, BL>), grid, dim3(HG_NT), 0, c->cur, a);
      } else if (h16)
        hipLaunchKernelGGL((gemm_h16_kernel<AL, BL, 1, 256, 64>), grid, dim3(HG_NT), 0, c->cur, a);
      else if (c->sw.gemm_h3 && m16) {
        // the same six plane products on the 16x16x32 MFMA (gemm_h3m.h)
        hipLaunchKernelGGL((gemm_h3m_kernel<AL, BL>), grid, dim3(HG_NT), 0, c->cur, a);
      } else if (c->sw.gemm_h3)
        // the same kernel with immediate-offset addressing (gemm_h3.h)
        hipLaunchKernelGGL((gemm_h3_kernel<AL, BL>), grid, dim3(HG_NT), 0, c->cur, a);
      else
        // SCH 1: fragment reads spread over the MFMA gaps (+2-4 % over the
        // burst schedule, bitwise equal; profiles/r3/gemmh_sched_c3.txt)
        hipLaunchKernelGGL((gemm_h_kernel<AL, BL, 3, 128, 32, 1>), grid, dim3(HG_NT), 0, c->cur, a);
      HIP_TRY(hipGetLastError());
      return h;
    }
  }
  if (nwe) throw einval("gemm %s: fused narrow weight gradient needs the twin path", name);
  if (p.splits == 1 && direct) {
    ee.out = direct;
    ee.out_split_stride = 0;
    p.direct = true;
  }
  GemmArgs g;
  g.A = A;
  g.B = B;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.kps = p.kps;
  g.xcd = c->sw.xcd;
  g.e = ee;
  dim3 grid(p.nt(N), p.mt(M), p.splits);
  // profile key "<kernel symbol>|<phase>": the symbol part matches rocprofv3's kernel names
  static const char* lay[2] = {"RK", "KR"};
  char key[112];
  if (bf || s3)  // one bf16 plane (bf16 configuration) or the exact three-plane split
    snprintf(key, sizeof key, "gemm_s3_kernel<%s,%s,NP=%d>|%s", lay[AL], lay[BL], bf ? 1 : 3,
             name);
  else
    snprintf(key, sizeof key, "gemm_f32_kernel<%s,%s,%d,%d,%d,%d>|%s", lay[AL], lay[BL],
             va ? 4 : 1, vb ? 4 : 1, p.bm, p.bn, name);
  // algorithmic bytes: each operand read once, the output (per split slab) written once
  ProfScope ps(c, key, 2.0 * M * N * (double)K,
               4.0 * ((double)M * K + (double)K * N + (double)M * N * p.splits));
  if (bf)
    hipLaunchKernelGGL((gemm_s3_kernel<AL, BL, 1>), grid, dim3(S3_NT), 0, c->cur, g);
  else if (s3)
    hipLaunchKernelGGL((gemm_s3_kernel<AL, BL, 3>), grid, dim3(S3_NT), 0, c->cur, g);
  else if (va && vb)
    gemm_dispatch<AL, BL, 4, 4>(p, grid, c->cur, g);
  else if (va)
    gemm_dispatch<AL, BL, 4, 1>(p, grid, c->cur, g);
  else if (vb)
    gemm_dispatch<AL, BL, 1, 4>(p, grid, c->cur, g);
  else
    gemm_dispatch<AL, BL, 1, 1>(p, grid, c->cur, g);
  HIP_TRY(hipGetLastError());
  return p;
}

// bf16 MFMA for the large GEMMs of a DDPG_BF16 context (thin / unaligned
// shapes stay on the exact-fp32 kernel)
static bool use_bf16(const ddpg_ctx* c, int M, int N, bool vec) {
  return c->cfg.dtype == DDPG_BF16 && vec && M >= 128 && N >= 128;
}

// fp32 contexts: the large GEMMs run fp32-accurate on the bf16 pipe
// (gemm_s3.h, three-plane split); env DDPG_GEMM=f32 keeps every GEMM on the
// fp32-input MFMA kernel.
static bool use_s3(const ddpg_ctx* c, int M, int N, bool vec) {
  return c->sw.gemm_s3 && c->cfg.dtype == DDPG_FP32 && vec && M >= 128 && N >= 128;
}

// Thin-K layers (thin_k.h) of fp32 contexts: K <= 64 and multiple of 8,
// 4-aligned widths / leading dims, 16-byte aligned operands (anything else goes
// through the GEMMs).  env DDPG_THINK=0 routes every such layer to the GEMMs.
static bool tk_valid(const TkPart& q) {
  // W[n][k] (w_nk) may have any stride: the kernel loads it as scalars then
  return q.K >= TK_KALIGN && q.K % TK_KALIGN == 0 && q.K <= TK_MAXK && q.ldx % 4 == 0 &&
         (q.w_nk || (q.ldw % 4 == 0 && aligned16(q.W))) && q.N % 4 == 0 && q.ldo % 4 == 0 &&
         aligned16(q.X) &&
         (!q.out || aligned16(q.out)) && (!q.bias || aligned16(q.bias)) &&
         (!q.aux || (q.ldaux % 4 == 0 && aligned16(q.aux)));
}

TkPart tk_part(const float* X, int ldx, int K, const float* W, int ldw, int w_nk, int N,
                      const float* bias, int act, float* out, int ldo) {
  TkPart p;
  memset(&p, 0, sizeof p);
  p.X = X;
  p.ldx = ldx;
  p.K = K;
  p.W = W;
  p.ldw = ldw;
  p.w_nk = w_nk;
  p.N = N;
  p.bias = bias;
  p.act = act;
  p.out = out;
  p.ldo = ldo;
  return p;
}

// Launch 1 .. TK_MAXP thin-K parts over M rows; returns the number of 64-row
// blocks (the row count of colsum partials), or 0 (nothing launched) when a
// layer is not eligible and the caller must use the GEMM.
// Launch the GEMMs queued under gemm_defer: one gemm_h16i_pack_kernel launch
// per GH_MAXP of them when they share a grid (DDPG_GEMM_PACK=0: one launch
// each, the same kernel body), in queue order.
void gemm_flush(ddpg_ctx* c) {
  std::vector<DeferredGemm> q;
  q.swap(c->deferred);
  size_t i = 0;
  while (i < q.size()) {
    size_t n = 1;
    while (c->sw.gemm_pack && i + n < q.size() && n < (size_t)GH_MAXP &&
           q[i + n].grid.x == q[i].grid.x && q[i + n].grid.y == q[i].grid.y)
      ++n;
    const bool f3 = c->hnp == 3;  // fp32 context: gemm_h3m (else gemm_h16i)
    if (n == 1) {
      ProfScope ps(c, q[i].key, q[i].flops, q[i].bytes);
      if (f3)
        hipLaunchKernelGGL((gemm_h3m_kernel<L_RK, L_KR>), q[i].grid, dim3(HG_NT), 0, c->cur, q[i].a);
      else
        hipLaunchKernelGGL((gemm_h16i_kernel<L_RK, L_KR>), q[i].grid, dim3(HG_NT), 0, c->cur,
                           q[i].a);
    } else {
      GemmHPack pk;
      double fl = 0, by = 0;
      // gemm_hw_pack_kernel (two 4-wave blocks per CU) when every part is a
      // full-tile forward layer (bias, elu; twin and / or fp32 out) of whole
      // 64-deep steps
      bool hw = c->sw.gemm_hw && !f3;
      for (size_t j = 0; j < n; ++j) {
        pk.p[j] = q[i + j].a;
        fl += q[i + j].flops;
        by += q[i + j].bytes;
        const GemmHArgs& a = q[i + j].a;
        const GemmEpi& e = a.e;
        hw = hw && a.M % 256 == 0 && a.N % HG_BN == 0 && a.kps == a.K && a.K % 64 == 0 &&
             !a.kpart && e.bias && e.act == 1 && e.post == 0 && !e.colsum && !e.proj_out &&
             !e.nw_out[0] && !e.nw_out[1] && !e.out_split_stride;
      }
      char key[128];
      snprintf(key, sizeof key, "%s<RK,KR,NP=%d>|%s",
               f3 ? "gemm_h3m_pack_kernel" : hw ? "gemm_hw_pack_kernel" : "gemm_h16i_pack_kernel",
               c->hnp, strchr(q[i].key, '|') + 1);
      ProfScope ps(c, key, fl, by);
      if (f3)
        hipLaunchKernelGGL((gemm_h3m_pack_kernel<L_RK, L_KR>), dim3(q[i].grid.x, q[i].grid.y, n),
                           dim3(HG_NT), 0, c->cur, pk);
      else if (hw)
        hipLaunchKernelGGL((gemm_hw_pack_kernel<L_RK, L_KR, HG_BN, 2, 64, 1>),
                           dim3(q[i].grid.x, q[i].grid.y, n), dim3(2 * HG_BN), 0, c->cur, pk);
      else
        hipLaunchKernelGGL((gemm_h16i_pack_kernel<L_RK, L_KR>), dim3(q[i].grid.x, q[i].grid.y, n),
                           dim3(HG_NT), 0, c->cur, pk);
    }
    HIP_TRY(hipGetLastError());
    i += n;
  }
}

int thin_k_launch(ddpg_ctx* c, const char* name, const TkPart* parts, int nparts, int M,
                  bool* dw_done) {
  if (dw_done) *dw_done = false;
  if (!c->sw.thin_k || nparts < 1 || nparts > TK_MAXP) return 0;
  TkPart pp[TK_MAXP];
  for (int i = 0; i < nparts; ++i) {
    pp[i] = parts[i];
    // K-padded to the 8-step of the kernel over zero-padded rows (the W rows
    // past K read are finite parameters of the next tensor, times zero)
    if (pp[i].K % TK_KALIGN && zero_padded(c, pp[i].X) && rup(pp[i].K, TK_KALIGN) <= pp[i].ldx &&
        pp[i].W >= c->dparams && pp[i].W < c->dparams + 2 * c->L.total)
      pp[i].K = rup(pp[i].K, TK_KALIGN);
    if (!tk_valid(pp[i])) return 0;
  }
  parts = pp;
  TkArgs a;
  memset(&a, 0, sizeof a);
  int nmax = 0;
  double flops = 0, bytes = 0;
  for (int i = 0; i < nparts; ++i) {
    a.p[i] = parts[i];
    const Twin to = act_twin(c, parts[i].out);
    if (to.p && !a.p[i].outh) {
      a.p[i].outh = to.p;
      a.p[i].hps = to.ps;
      a.p[i].hnp = c->hnp;
    }
    nmax = std::max(nmax, parts[i].N);
    flops += 2.0 * M * parts[i].N * (double)parts[i].K;
    bytes += 4.0 * ((double)M * parts[i].K + (double)parts[i].K * parts[i].N +
                    (double)M * parts[i].N);
  }
  a.M = M;
  const int mt = ceil_div(M, TK_ROWS);
  const int nc = ceil_div(nmax, TK_COLS);
  // row tiles per block: the fewest that keep the grid within one round of
  // the device's block slots (c->tk_slots: CUs x the TK_LDS-byte blocks one
  // CU's LDS holds -- 256 x 2 on MI355X), so that a block stages its W panel
  // once for several row tiles and overlaps the next X tile's loads with its
  // stores (env DDPG_TK_RPB=n forces n; 1 = one tile)
  int rpb = 1;
  if (c->sw.tk_rpb > 0) {
    rpb = std::min(c->sw.tk_rpb, mt);
  } else {
    while (rpb < mt && nc * nparts * ceil_div(mt, rpb) > c->tk_slots) ++rpb;
  }
  a.mt = mt;
  a.rpb = rpb;
  // the forward / backward forms when every part is one (thin_k.h)
  bool fwd = c->sw.tk_fwd && M % TK_ROWS == 0, bwd = fwd;
  for (int i = 0; i < nparts; ++i) {
    const TkPart& q = a.p[i];
    const bool full = q.N % TK_COLS == 0 && q.ldo % 8 == 0 &&
                      (!q.outh || (q.hps % 8 == 0 && ((uintptr_t)q.outh & 15) == 0));
    fwd = fwd && full && q.bias && q.act == 1 && q.outh && !q.aux && !q.colsum;
    bwd = bwd && full && !q.bias && q.act == 0 && q.aux && q.colsum && q.ldaux % 4 == 0;
  }
  // a fused weight gradient (TkPart.dw) needs the aux rows (backward or
  // generic form) and full row tiles; a part that cannot carry it runs
  // unfused (the caller sees *dw_done false and computes it elsewhere)
  bool dw_all = true;
  for (int i = 0; i < nparts; ++i)
    if (a.p[i].dw && !(!fwd && a.p[i].aux && M % TK_ROWS == 0 && a.p[i].dw_k >= 1 &&
                       a.p[i].dw_k <= a.p[i].K && a.p[i].K <= 32)) {
      a.p[i].dw = nullptr;
      dw_all = false;
    }
  char key[96];
  snprintf(key, sizeof key, "thin_k_kernel%s|%s", fwd ? "<FWD>" : bwd ? "<BWD>" : "", name);
  if (c->sw.prof_shapes)
    snprintf(key + strlen(key), sizeof key - strlen(key), " %dp %dx%dx%d", nparts, M, parts[0].N,
             parts[0].K);
  ProfScope ps(c, key, flops, bytes);
  const dim3 grid(nc, ceil_div(mt, rpb), nparts);
  bool dw = false;
  for (int i = 0; i < nparts; ++i) dw = dw || a.p[i].dw;
  if (fwd)
    hipLaunchKernelGGL(thin_k_kernel<1>, grid, dim3(TK_NT), 0, c->cur, a);
  else if (bwd && dw)
    hipLaunchKernelGGL((thin_k_kernel<2, true>), grid, dim3(TK_NT), 0, c->cur, a);
  else if (bwd)
    hipLaunchKernelGGL(thin_k_kernel<2>, grid, dim3(TK_NT), 0, c->cur, a);
  else if (dw)
    hipLaunchKernelGGL((thin_k_kernel<0, true>), grid, dim3(TK_NT), 0, c->cur, a);
  else
    hipLaunchKernelGGL(thin_k_kernel<0>, grid, dim3(TK_NT), 0, c->cur, a);
  HIP_TRY(hipGetLastError());
  if (dw_done) *dw_done = dw_all && dw;
  return mt;
}

// Weight gradient dW[M][N] = A^T . B over K = B rows (A [K][lda] M columns,
// B [K][ldb] N columns; split-K slabs [split][M][N] or `direct`): on the
// skinny kernel (skinny.h) when one side is at most 64 wide and the other a
// multiple of 4 (>= 128), with the narrow operand's row holding every column
// its NG-wide tiles read; otherwise on the GEMMs.
GemmPlan wgrad_launch(ddpg_ctx* c, const float* A, int lda, const float* B, int ldb, int M,
                             int N, int K, float* slab, int cap, float* direct) {
  const bool a_narrow = M <= SK_NMAX && N >= 128;
  const bool b_narrow = N <= SK_NMAX && M >= 128 && !a_narrow;
  const float* nar = a_narrow ? A : B;
  const int ldn = a_narrow ? lda : ldb, nn = a_narrow ? M : N;
  const int ldw = a_narrow ? ldb : lda, nw = a_narrow ? N : M;
  // 16 narrow columns per wave above 16 (one 128 KB reduction: 1 block per
  // CU, 256 blocks); 8 at or below (64 KB, 2 blocks per CU, 512 blocks) --
  // measured, profiles/r3/skinny_variants.txt
  const int ng = (nn > 16 && rup(nn, 16) <= ldn) ? 16 : 8;
  const int ntn = ceil_div(std::max(nn, 1), ng);
  if (c->sw.skinny && (a_narrow || b_narrow) && nw % 4 == 0 && ldw % 4 == 0 &&
      ntn * ng <= ldn && aligned16(a_narrow ? B : A)) {
    GemmPlan p;
    const int ntw = ceil_div(nw, SK_WT), tiles = ntw * ntn;
    int splits = std::min(cap, std::max(1, (ng == 8 ? 512 : 256) / tiles));
    int kc = rup(ceil_div(K, splits), SK_WAVES);
    splits = ceil_div(K, kc);
    p.splits = splits;
    SkArgs a;
    a.N = nar;
    a.ldn = ldn;
    a.nn = nn;
    a.W = a_narrow ? B : A;
    a.ldw = ldw;
    a.nw = nw;
    a.B = K;
    a.kc = kc;
    a.ntw = ntw;
    a.ntn = ntn;
    a.narrow_rows = a_narrow ? 1 : 0;
    if (splits == 1 && direct) {
      a.out = direct;
      a.split_stride = 0;
      p.direct = true;
    } else {
      a.out = slab;
      a.split_stride = (long long)M * N;
    }
    ProfScope ps(c, "skinny_wgrad_kernel|wgrad", 2.0 * M * N * (double)K,
                 4.0 * ((double)K * (M + N) + (double)M * N * splits));
    // narrow rows through LDS (skinny.h, NL) when the split's rows fit
    const bool nl = c->sw.skinny_nl && kc <= sk_nl_rows(ng);
    const dim3 grid(tiles * splits);
    if (ng == 8) {
      if (nl)
        hipLaunchKernelGGL((skinny_wgrad_kernel<8, SK_R, true>), grid, dim3(SK_NT), sk_lds_bytes(8),
                           c->cur, a);
      else
        hipLaunchKernelGGL((skinny_wgrad_kernel<8, SK_R, false>), grid, dim3(SK_NT),
                           sk_lds_bytes(8), c->cur, a);
    } else {
      if (nl)
        hipLaunchKernelGGL((skinny_wgrad_kernel<16, SK_R, true>), grid, dim3(SK_NT),
                           sk_lds_bytes(16), c->cur, a);
      else
        hipLaunchKernelGGL((skinny_wgrad_kernel<16, SK_R, false>), grid, dim3(SK_NT),
                           sk_lds_bytes(16), c->cur, a);
    }
    HIP_TRY(hipGetLastError());
    return p;
  }
  GemmEpi e = epi_none();
  e.out = slab;
  e.ldo = N;
  e.out_split_stride = (long long)M * N;
  return gemm_launch<L_KR, L_KR>(c, "wgrad", A, lda, B, ldb, M, N, K, e, 0, cap, direct);
}

// ddpg_create's GEMM part: the split-K caps of the weight gradients (the slab
// sizes), the small-M plan's partial buffers and ticket segments, and the
// dynamic-LDS attributes of the skinny weight-gradient kernels.
void gemm_setup(ddpg_ctx* c) {
  if (const char* mb = getenv("DDPG_GEMM_MIN_BLOCKS")) g_min_blocks = std::max(1, atoi(mb));
  c->split_cap_W1 = make_plan(c->S, c->AH1, c->Bmax, 0).splits;
  c->split_cap_W2 = make_plan(c->AH1, c->AH2, c->Bmax, 0).splits;
  c->split_cap_W3 = make_plan(c->AH2, c->A, c->Bmax, 0).splits;
  c->split_cap_Ws = make_plan(c->S, c->CH1, c->Bmax, 0).splits;
  c->split_cap_Wa = make_plan(c->A, c->CH1, c->Bmax, 0).splits;
  c->split_cap_Wh = make_plan(2 * c->CH1, c->CH2, c->Bmax, 0).splits;
  if (c->cfg.dtype == DDPG_BF16) {  // the 256 x 256-tile kernel splits finer
    auto cap256 = [&](int M, int N) {
      return (M % H2_BM || N % H2_BN) ? 1 : std::max(1, 256 / ((M / H2_BM) * (N / H2_BN)));
    };
    c->split_cap_W2 = std::max(c->split_cap_W2, cap256(c->AH1, c->AH2));
    c->split_cap_Wh = std::max(c->split_cap_Wh, cap256(2 * c->CH1, c->CH2));
  }
  if (c->hnp && c->sw.kcomb) {
    // a combined launch has S x tiles < 256 + kc_blocks blocks of BM x 128
    // partials; two buffers suffice on one stream, eight cover the
    // concurrent branches of DDPG_PAR=1
    const int BMh = c->hnp == 1 ? 256 : 128;
    c->kc_rot = c->par ? 8 : 2;
    c->kc_part_n = (size_t)(256 + c->sw.kc_blocks) * BMh * HG_BN;
    HIP_TRY(hipMalloc(&c->kc_part, c->kc_rot * c->kc_part_n * sizeof(float)));
    HIP_TRY(hipMalloc(&c->kc_ticket, (size_t)c->kc_rot * kKcTickets * sizeof(unsigned)));
    HIP_TRY(hipMemset(c->kc_ticket, 0, (size_t)c->kc_rot * kKcTickets * sizeof(unsigned)));
  }
  HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<8, SK_R, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(8)));
  HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<16, SK_R, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(16)));
  HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<8, SK_R, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(8)));
  HIP_TRY(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<16, SK_R, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(16)));
}

// the layouts the learner uses (RK x KR forward, RK x RK dX, KR x KR weight gradients)
template bool gemm_h_ok<L_RK, L_KR>(const ddpg_ctx*, const float*, int, const float*, int, int, int,
                                    int, int, int*);
template bool gemm_h_ok<L_RK, L_RK>(const ddpg_ctx*, const float*, int, const float*, int, int, int,
                                    int, int, int*);
template bool gemm_h_ok<L_KR, L_KR>(const ddpg_ctx*, const float*, int, const float*, int, int, int,
                                    int, int, int*);
template GemmPlan gemm_launch<L_RK, L_KR>(ddpg_ctx*, const char*, const float*, int, const float*,
                                          int, int, int, int, const GemmEpi&, int, int, float*);
template GemmPlan gemm_launch<L_RK, L_RK>(ddpg_ctx*, const char*, const float*, int, const float*,
                                          int, int, int, int, const GemmEpi&, int, int, float*);
template GemmPlan gemm_launch<L_KR, L_KR>(ddpg_ctx*, const char*, const float*, int, const float*,
                                          int, int, int, int, const GemmEpi&, int, int, float*);
