// Synchronous data parallelism (replacing the reference's TF
// parameter server, ddpg.py:168-174): the RCCL exchange on the comm stream,
// the stats all-gather, and the communicator ABI.  DESIGN.md §6.
#include "ctx.h"

// Data-parallel stats (world > 1): all[w] = rank w's {q_max, loss share};
// max and an ordered sum, identical on every rank.
__global__ void stats_reduce_kernel(const float* __restrict__ all, int world,
                                    float* __restrict__ stats, double* __restrict__ acc) {
  if (threadIdx.x != 0) return;
  float qm = all[0], ls = all[1];
  for (int w = 1; w < world; ++w) {
    qm = fmaxf(qm, all[2 * w]);
    ls = __fadd_rn(ls, all[2 * w + 1]);
  }
  stats[0] = qm;
  stats[1] = ls;
  if (acc) {
    acc[0] += (double)qm;
    acc[1] += (double)ls;
    acc[2] += 1.0;
  }
}

// Test hook of the data-parallel ordering (env DDPG_TEST_CS_SPIN=us; the
// comm stream, ahead of a collective group): every block waits `us`
// microseconds of wall clock (100 MHz s_memrealtime), then the grid doubles
// the two gradient ranges the group exchanges (exact in fp32).  A reader not
// ordered behind the comm stream would see the undoubled values.
__global__ void cs_spin_scale_kernel(float* b0, long long n0, float* b1, long long n1, int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * (unsigned long long)us)
    __builtin_amdgcn_s_sleep(8);
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long long i = i0; i < n0; i += stride) b0[i] = 2.f * b0[i];
  for (long long i = i0; i < n1; i += stride) b1[i] = 2.f * b1[i];
}

// bf16 configuration's exchange ("bf16 with fp32
// accumulation"): an fp32 reduce-scatter (each rank sums its slice of the
// ranks' fp32 gradients in fp32), the slice rounded once to bf16, a bf16
// all-gather, widened back into the fp32 gradient buffer for Adam.  Every
// rank ends with the same bits (the owner's rounding), the sum carries one
// bf16 rounding whatever N, and the links move 4 + 2 B per element per
// (N-1)/N instead of 8 (fp32 all-reduce).
__global__ void f32_to_bf16_kernel(const float* __restrict__ x, long long n,
                                   __bf16* __restrict__ y) {
  const long long i0 = 4 * ((long long)blockIdx.x * blockDim.x + threadIdx.x);
  const long long stride = 4ll * gridDim.x * blockDim.x;
  for (long long i = i0; i < n; i += stride) {
    if (i + 4 <= n) {
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      y[i] = (__bf16)v.x;
      y[i + 1] = (__bf16)v.y;
      y[i + 2] = (__bf16)v.z;
      y[i + 3] = (__bf16)v.w;
    } else {
      for (long long j = i; j < n; ++j) y[j] = (__bf16)x[j];
    }
  }
}
__global__ void bf16_to_f32_kernel(const __bf16* __restrict__ y, long long n,
                                   float* __restrict__ x) {
  const long long i0 = 4 * ((long long)blockIdx.x * blockDim.x + threadIdx.x);
  const long long stride = 4ll * gridDim.x * blockDim.x;
  for (long long i = i0; i < n; i += stride) {
    if (i + 4 <= n)
      *reinterpret_cast<float4*>(x + i) =
          make_float4((float)y[i], (float)y[i + 1], (float)y[i + 2], (float)y[i + 3]);
    else
      for (long long j = i; j < n; ++j) x[j] = (float)y[j];
  }
}

static void nccl_try(ncclResult_t r) {
  if (r != ncclSuccess) throw DdpgError(DDPG_ECOMM, ncclGetErrorString(r));
}

// `to` waits for the work queued so far on `from` (comm-stream events cev)
static void cs_link(ddpg_ctx* c, int ev, hipStream_t from, hipStream_t to) {
  if (from == to) return;
  HIP_TRY(hipEventRecord(c->cev[ev], from));
  HIP_TRY(hipStreamWaitEvent(to, c->cev[ev], 0));
}

// In-place RCCL sums of up to 2 disjoint ranges of the flat grad buffer, on
// the comm stream after the work queued so far on c->cur (one group: one
// launch).  The caller joins cs back before the gradients are read.
// with_stats: the all-gather of the step's {q_max, loss} joins the same group
// (one collective launch, one latency on the critical path instead of two);
// stats_allreduce_on_cs then only reduces the gathered values.
// window (profiling only): open an exchange-overlap record on the producing
// stream, closed by the next join_cs -- the compute that stream runs between
// issuing this exchange and waiting for it (bench.py's projected scaling).
void allreduce_on_cs(ddpg_ctx* c, int ev, const char* name, float* b0, size_t n0,
                            float* b1, size_t n1, bool with_stats,
                            const char* window) {
  if (!c->comm) return;
  cs_link(c, ev, c->cur, c->cs);
  const hipStream_t prev = c->cur;
  if (window && c->prof) {
    ProfRec rec{window, ev_get(c), ev_get(c), 0.0, (double)n0 * 4.0};
    HIP_TRY(hipEventRecord(rec.e0, prev));
    c->prof_recs.push_back(rec);
    c->win_open.push_back((int)c->prof_recs.size() - 1);
  }
  c->cur = c->cs;
  if (c->test_cs_spin) {
    // test hook: the exchanged ranges doubled after a delay, on cs ahead of
    // the group -- a consumer not ordered behind cs reads them undoubled
    hipLaunchKernelGGL(cs_spin_scale_kernel, dim3(256), dim3(256), 0, c->cs, b0, (long long)n0,
                       b1, (long long)n1, c->test_cs_spin);
    HIP_TRY(hipGetLastError());
  }
  // bf16 configuration: fp32 reduce-scatter + bf16 all-gather
  const bool half = c->xbuf != nullptr;
  const int N = c->cworld;
  float* const bs[2] = {b0, b1};
  const size_t ns[2] = {n0, n1};
  // per range: m = the largest multiple of N in n (reduce-scattered, chunk
  // elements per rank), the n - m tail elements all-reduced in fp32
  size_t m[2], chunk[2];
  __bf16* h[2] = {nullptr, nullptr};
  float* rs[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; ++k) {
    m[k] = ns[k] - ns[k] % N;
    chunk[k] = m[k] / N;
  }
  if (half) {
    h[0] = c->xbuf;
    h[1] = c->xbuf + n0;
    rs[0] = c->xrs;
    rs[1] = c->xrs + ((chunk[0] + 3) & ~(size_t)3);  // 16-B aligned (float4 reads)
  }
  auto blocks = [](size_t n) { return (int)std::min<size_t>(2048, (n + 1023) / 1024); };
  {
    ProfScope ps(c, name, 0,
                 (double)(n0 + n1) * (half ? 3.0 : 4.0) + (with_stats ? 8.0 * c->cworld : 0.0));
    // the group is closed on every path: a call that fails inside it still
    // runs ncclGroupEnd before the error propagates, so the thread's group
    // depth is back to zero for the caller's next (eager) step
    nccl_try(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    for (int k = 0; k < 2 && r == ncclSuccess; ++k) {
      if (!ns[k]) continue;
      if (!half) {
        r = ncclAllReduce(bs[k], bs[k], ns[k], ncclFloat, ncclSum, c->comm, c->cs);
        continue;
      }
      if (chunk[k])
        r = ncclReduceScatter(bs[k], rs[k], chunk[k], ncclFloat, ncclSum, c->comm, c->cs);
      if (r == ncclSuccess && ns[k] > m[k])
        r = ncclAllReduce(bs[k] + m[k], bs[k] + m[k], ns[k] - m[k], ncclFloat, ncclSum, c->comm,
                          c->cs);
    }
    if (r == ncclSuccess && with_stats)
      r = ncclAllGather(c->dstats, c->dstats_all, 2, ncclFloat, c->comm, c->cs);
    ncclResult_t re = ncclGroupEnd();
    nccl_try(r);
    nccl_try(re);
    if (half && (chunk[0] || chunk[1])) {
      // this rank's fp32 sums rounded once, into its slot of the gather
      for (int k = 0; k < 2; ++k)
        if (chunk[k]) {
          hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(blocks(chunk[k])), dim3(256), 0, c->cs,
                             rs[k], (long long)chunk[k], h[k] + (size_t)c->crank * chunk[k]);
          HIP_TRY(hipGetLastError());
        }
      nccl_try(ncclGroupStart());
      for (int k = 0; k < 2 && r == ncclSuccess; ++k)
        if (chunk[k])
          r = ncclAllGather(h[k] + (size_t)c->crank * chunk[k], h[k], chunk[k], ncclBfloat16,
                            c->comm, c->cs);
      re = ncclGroupEnd();
      nccl_try(r);
      nccl_try(re);
      for (int k = 0; k < 2; ++k)
        if (chunk[k]) {
          hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(blocks(m[k])), dim3(256), 0, c->cs, h[k],
                             (long long)m[k], bs[k]);
          HIP_TRY(hipGetLastError());
        }
    }
  }
  c->cur = prev;
}

// the logged stats of a data-parallel step are the
// global-batch ones (ddpg.py:102-103) -- max over ranks of max(Q) and the sum
// of the ranks' loss shares (each already scaled by 1/B_global).  One
// all-gather of every rank's {q_max, loss}, then an ordered reduction that
// every rank computes identically; it also feeds the running sums.  On the
// comm stream, after the critic all-reduce.
void stats_allreduce_on_cs(ddpg_ctx* c, bool gathered) {
  if (!c->comm) return;
  const hipStream_t prev = c->cur;
  c->cur = c->cs;
  {
    ProfScope ps(c, "rccl_stats", 0, gathered ? 0.0 : 8.0 * c->cworld);
    if (!gathered)
      nccl_try(ncclAllGather(c->dstats, c->dstats_all, 2, ncclFloat, c->comm, c->cs));
    hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(64), 0, c->cs, c->dstats_all, c->cworld,
                       c->dstats, c->dacc);
    HIP_TRY(hipGetLastError());
  }
  c->cur = prev;
}

// the consumer stream (c->cur) waits for every collective queued on cs
void join_cs(ddpg_ctx* c, int ev) {
  if (!c->comm) return;
  for (int w : c->win_open)  // close the exchange-overlap windows on the consumer stream
    HIP_TRY(hipEventRecord(c->prof_recs[w].e1, c->cur));
  c->win_open.clear();
  cs_link(c, ev, c->cs, c->cur);
}

extern "C" {

// ---------------------------------------------------------------- comm
// comm stream, its events and the stats all-gather buffer for a communicator
// of `cworld` ranks
static void comm_setup(ddpg_ctx* c, int cworld) {
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (!c->dstats_all) HIP_TRY(hipMalloc(&c->dstats_all, 2 * (size_t)cworld * sizeof(float)));
  if (!c->cs) HIP_TRY(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  if (c->cfg.dtype == DDPG_BF16 && !c->xbuf) {
    HIP_TRY(hipMalloc(&c->xbuf, (size_t)c->L.total * sizeof(__bf16)));
    // the reduce-scatter slices of one call's ranges: at most L.total / cworld
    // floats (+ alignment); L.total covers every communicator size
    HIP_TRY(hipMalloc(&c->xrs, ((size_t)c->L.total + 8) * sizeof(float)));
  }
  for (auto& ev : c->cev)
    if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
}

int ddpg_comm_unique_id(char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    g_err = ncclGetErrorString(r);
    return DDPG_ECOMM;
  }
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out128, &id, 128);
  return DDPG_OK;
}

int ddpg_comm_init(ddpg_ctx* c, const char* id128, int world, int rank) {
  return guard(c, [&] {
    if (world != c->world || rank != c->rank)
      throw einval("comm (%d/%d) != cfg (%d/%d)", rank, world, c->rank, c->world);
    if (!id128) throw einval("null unique id");
    if (c->comm) throw DdpgError(DDPG_ESTATE, "communicator already initialised");
    // world == 1 makes a 1-rank communicator: the data-parallel exchange then
    // runs (as an identity) through the same RCCL call sites as world > 1
    ncclUniqueId id;
    memcpy(&id, id128, 128);
    comm_setup(c, world);
    nccl_try(ncclCommInitRank(&c->comm, world, id, rank));
    c->cworld = world;
    c->crank = rank;
  });
}

int ddpg_comm_init_proxy(ddpg_ctx* c) {
  return guard(c, [&] {
    if (c->comm) throw DdpgError(DDPG_ESTATE, "communicator already initialised");
    ncclUniqueId id;
    nccl_try(ncclGetUniqueId(&id));
    comm_setup(c, 1);
    nccl_try(ncclCommInitRank(&c->comm, 1, id, 0));
    c->cworld = 1;
    c->crank = 0;
  });
}

}  // extern "C"
