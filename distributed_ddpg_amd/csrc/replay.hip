// The device replay ring (ReplayBuffer, replay_buffer.py:10-51) and the host
// MT19937 random.sample restatement behind sample_batch.  DESIGN.md §3.
#include "ctx.h"

// Row gather of one ring plane as raw 32-bit words (host sample_batch path:
// the rows keep the ring's precision; row_bytes is a multiple of 4).
__global__ void gather_bytes_kernel(const int* __restrict__ slots, int B,
                                    const unsigned char* __restrict__ src,
                                    unsigned char* __restrict__ dst, long long row_bytes) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const long long words = row_bytes >> 2;
  for (int b = wave; b < B; b += nwaves) {
    const unsigned* ps = (const unsigned*)(src + (size_t)slots[b] * row_bytes);
    unsigned* pd = (unsigned*)(dst + (size_t)b * row_bytes);
    for (long long j = lane; j < words; j += 64) pd[j] = ps[j];
  }
}


extern "C" {

// ---------------------------------------------------------------- sampler
struct ddpg_sampler {
  Sampler s;
  explicit ddpg_sampler(int64_t seed) : s(seed) {}
};

int ddpg_sampler_create(int64_t seed, ddpg_sampler** out) {
  if (!out) return DDPG_EINVAL;
  *out = new ddpg_sampler(seed);
  return DDPG_OK;
}
void ddpg_sampler_destroy(ddpg_sampler* s) { delete s; }
int ddpg_sampler_sample(ddpg_sampler* s, int64_t n, int k, int64_t* out) {
  if (!s || !out || s->s.sample(n, k, out) != 0) {
    g_err = "sample larger than population or is negative";
    return DDPG_EINVAL;
  }
  return DDPG_OK;
}
int ddpg_sampler_getrandbits32(ddpg_sampler* s, uint32_t* out, int n) {
  if (!s || !out || n < 0) return DDPG_EINVAL;
  for (int i = 0; i < n; ++i) out[i] = s->s.rng.genrand_uint32();
  return DDPG_OK;
}

// ---------------------------------------------------------------- replay
static constexpr int kStageRows = 1024;

static int replay_create_impl(int device, int S, int A, int64_t cap, int64_t seed, int flags,
                              ddpg_replay** out) {
  if (!out) return DDPG_EINVAL;
  ddpg_replay* rb = new ddpg_replay(seed);
  int rc = rguard(rb, [&] {
    if (S <= 0 || A <= 0 || cap <= 0) throw einval("bad replay dims S=%d A=%d cap=%lld", S, A,
                                                   (long long)cap);
    if (flags & ~DDPG_REPLAY_F64) throw einval("bad replay flags %d", flags);
    rb->device = device;
    rb->S = S;
    rb->A = A;
    rb->cap = cap;
    rb->f64 = (flags & DDPG_REPLAY_F64) != 0;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&rb->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&rb->last_read, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&rb->written, hipEventDisableTiming));
    const char* ra_env = getenv("DDPG_RING_ARGS");
    rb->args_flush = !(ra_env && strcmp(ra_env, "0") == 0);
    const size_t c = (size_t)cap, es = rb->es();
    void *ps, *ps2, *pr;
    HIP_TRY(hipMalloc(&ps, c * S * es));
    HIP_TRY(hipMalloc(&ps2, c * S * es));
    HIP_TRY(hipMalloc(&pr, c * es));
    if (rb->f64) {
      rb->rsd = (double*)ps;
      rb->rs2d = (double*)ps2;
      rb->rrd = (double*)pr;
    } else {
      rb->rs = (float*)ps;
      rb->rs2 = (float*)ps2;
      rb->rr = (float*)pr;
    }
    HIP_TRY(hipMalloc(&rb->ra, c * A * 4));
    HIP_TRY(hipMalloc(&rb->rt, c * 4));
    rb->st_s.resize((size_t)kStageRows * S * es);
    rb->st_s2.resize((size_t)kStageRows * S * es);
    rb->st_r.resize((size_t)kStageRows * es);
    rb->st_a.resize((size_t)kStageRows * A);
    rb->st_t.resize(kStageRows);
  });
  if (rc != DDPG_OK) {
    ddpg_replay_destroy(rb);
    *out = nullptr;
    return rc;
  }
  *out = rb;
  return DDPG_OK;
}

int ddpg_replay_create(int device, int S, int A, int64_t cap, int64_t seed, ddpg_replay** out) {
  return replay_create_impl(device, S, A, cap, seed, 0, out);
}

int ddpg_replay_create_ex(int device, int S, int A, int64_t cap, int64_t seed, int flags,
                          ddpg_replay** out) {
  return replay_create_impl(device, S, A, cap, seed, flags, out);
}

int ddpg_replay_is_f64(ddpg_replay* rb) { return rb && rb->f64 ? 1 : 0; }

void ddpg_replay_destroy(ddpg_replay* rb) {
  if (!rb) return;
  (void)hipSetDevice(rb->device);
  if (rb->stream) (void)hipStreamSynchronize(rb->stream);
  if (rb->written) (void)hipEventSynchronize(rb->written);
  for (void* p : {(void*)rb->rs, (void*)rb->rs2, (void*)rb->rr, (void*)rb->rsd, (void*)rb->rs2d,
                  (void*)rb->rrd, (void*)rb->ra, (void*)rb->rt, (void*)rb->d_slots,
                  (void*)rb->d_tmp})
    if (p) (void)hipFree(p);
  if (rb->stream) (void)hipStreamDestroy(rb->stream);
  if (rb->last_read) (void)hipEventDestroy(rb->last_read);
  if (rb->written) (void)hipEventDestroy(rb->written);
  delete rb;
}

const char* ddpg_replay_last_error(ddpg_replay* rb) { return rb ? rb->err.c_str() : ""; }

// copy n consecutive insertions starting at insertion index `first` into the
// ring; s, s2, r are already in the ring's precision (rb->es() bytes each)
static void ring_write(ddpg_replay* rb, int64_t first, int n, const void* s, const float* a,
                       const void* r, const float* t, const void* s2) {
  const size_t es = rb->es(), S = rb->S, A = rb->A;
  const unsigned char* bs = (const unsigned char*)s;
  const unsigned char* bs2 = (const unsigned char*)s2;
  const unsigned char* br = (const unsigned char*)r;
  int done = 0;
  while (done < n) {
    const int64_t slot = (first + done) % rb->cap;
    const size_t run = (size_t)std::min<int64_t>(n - done, rb->cap - slot);
    HIP_TRY(hipMemcpyAsync(rb->ps() + slot * S * es, bs + done * S * es, run * S * es,
                           hipMemcpyHostToDevice, rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->ps2() + slot * S * es, bs2 + done * S * es, run * S * es,
                           hipMemcpyHostToDevice, rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->pr() + slot * es, br + done * es, run * es, hipMemcpyHostToDevice,
                           rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->ra + slot * A, a + done * A, run * A * 4, hipMemcpyHostToDevice,
                           rb->stream));
    HIP_TRY(hipMemcpyAsync(rb->rt + slot, t + done, run * 4, hipMemcpyHostToDevice, rb->stream));
    done += (int)run;
  }
}

// A few staged rows written into the ring by one block, the rows in the
// kernel arguments ([s rows][s2 rows][r][a][t] as 32-bit words, s / s2 / r in
// the ring's precision): the host staging is free again when the launch call
// returns, so the flush needs no host wait.
constexpr int kRingArgWords = 512;
struct RingRowsIn {
  unsigned w[kRingArgWords];
};
__global__ __launch_bounds__(256) void ring_rows_kernel(RingRowsIn in, int n, long long first,
                                                        long long cap, int sw, int rw, int A,
                                                        unsigned* __restrict__ ps,
                                                        unsigned* __restrict__ ps2,
                                                        unsigned* __restrict__ pr,
                                                        unsigned* __restrict__ pa,
                                                        unsigned* __restrict__ pt) {
  // sw / rw: words per s row / per r value; A words per a row; 1 per t
  const int seg[5] = {sw, sw, rw, A, 1};
  unsigned* dst[5] = {ps, ps2, pr, pa, pt};
  int off = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int per = seg[q];
    for (int i = threadIdx.x; i < n * per; i += 256) {
      const int row = i / per;
      const long long slot = (first + row) % cap;
      dst[q][slot * per + (i - row * per)] = in.w[off + i];
    }
    off += n * per;
  }
}

// rb->stream's next ring access after the last kernel-argument flush, which
// may have run on a learner's stream
static void ring_join(ddpg_replay* rb) {
  if (rb->written_rec && rb->written_by) HIP_TRY(hipStreamWaitEvent(rb->stream, rb->written, 0));
}

extern "C++" {  // declared in ctx.h (C++ linkage)
void replay_flush(ddpg_replay* rb, hipStream_t on, uint64_t by) {
  if (rb->st_n == 0) return;
  const size_t es = rb->es(), S = rb->S, A = rb->A, n = (size_t)rb->st_n;
  const size_t sw = S * es / 4, rw = es / 4;
  if (rb->args_flush && n * (2 * sw + rw + A + 1) <= (size_t)kRingArgWords) {
    // the reading learner's own stream when known: its previous gather is
    // then ordered before these writes, and its next one after them
    const hipStream_t st = on ? on : rb->stream;
    if (rb->last_read) HIP_TRY(hipStreamWaitEvent(st, rb->last_read, 0));
    RingRowsIn in;
    unsigned char* b = reinterpret_cast<unsigned char*>(in.w);
    memcpy(b, rb->st_s.data(), n * S * es);
    b += n * S * es;
    memcpy(b, rb->st_s2.data(), n * S * es);
    b += n * S * es;
    memcpy(b, rb->st_r.data(), n * es);
    b += n * es;
    memcpy(b, rb->st_a.data(), n * A * 4);
    b += n * A * 4;
    memcpy(b, rb->st_t.data(), n * 4);
    hipLaunchKernelGGL(ring_rows_kernel, dim3(1), dim3(256), 0, st, in, (int)n,
                       (long long)rb->st_first, (long long)rb->cap, (int)sw, (int)rw, (int)A,
                       (unsigned*)rb->ps(), (unsigned*)rb->ps2(), (unsigned*)rb->pr(), (unsigned*)rb->ra,
                       (unsigned*)rb->rt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(rb->written, st));
    rb->written_by = on ? by : 0;
    rb->written_rec = true;
    rb->st_n = 0;
    return;
  }
  if (rb->last_read) HIP_TRY(hipStreamWaitEvent(rb->stream, rb->last_read, 0));
  ring_join(rb);
  ring_write(rb, rb->st_first, rb->st_n, rb->st_s.data(), rb->st_a.data(), rb->st_r.data(),
             rb->st_t.data(), rb->st_s2.data());
  HIP_TRY(hipStreamSynchronize(rb->stream));  // staging is reused after this
  rb->st_n = 0;
}
}  // extern "C++"

extern "C++" {
// n host values of type T into dst in the ring's precision (float or double)
template <class T>
static void to_ring(const ddpg_replay* rb, const T* src, size_t n, unsigned char* dst) {
  if (rb->f64) {
    double* d = (double*)dst;
    for (size_t i = 0; i < n; ++i) d[i] = (double)src[i];
  } else {
    float* d = (float*)dst;
    for (size_t i = 0; i < n; ++i) d[i] = (float)src[i];
  }
}

// ReplayBuffer.add for n rows whose s, s2, r are float (T = float) or float64
// (T = double); converted to the ring's precision on the host.
template <class T>
static void replay_add_impl(ddpg_replay* rb, const T* s, const float* a, const T* r,
                            const uint8_t* t, const T* s2, int n) {
  if (n < 0) throw einval("negative row count");
  if (n > 0 && (!s || !a || !r || !t || !s2)) throw einval("null row array");
  HIP_TRY(hipSetDevice(rb->device));
  const size_t S = rb->S, A = rb->A, es = rb->es();
  if (n >= kStageRows) {  // bulk insert
    replay_flush(rb);
    if (rb->last_read) HIP_TRY(hipStreamWaitEvent(rb->stream, rb->last_read, 0));
    ring_join(rb);
    // only the last `cap` rows can survive; skip the ones that would be overwritten
    const int64_t skip = n > rb->cap ? n - rb->cap : 0;
    const size_t m = (size_t)(n - skip);
    std::vector<float> tf(m);
    for (size_t i = 0; i < m; ++i) tf[i] = t[skip + i] ? 1.f : 0.f;
    const bool same = (sizeof(T) == es);  // caller's arrays already in ring precision
    std::vector<unsigned char> cs, cs2, cr;
    const void *ps = s + skip * S, *ps2 = s2 + skip * S, *pr = r + skip;
    if (!same) {
      cs.resize(m * S * es);
      cs2.resize(m * S * es);
      cr.resize(m * es);
      to_ring(rb, s + skip * S, m * S, cs.data());
      to_ring(rb, s2 + skip * S, m * S, cs2.data());
      to_ring(rb, r + skip, m, cr.data());
      ps = cs.data();
      ps2 = cs2.data();
      pr = cr.data();
    }
    ring_write(rb, rb->total + skip, (int)m, ps, a + skip * A, pr, tf.data(), ps2);
    HIP_TRY(hipStreamSynchronize(rb->stream));
    rb->total += n;
    rb->count = std::min<int64_t>(rb->total, rb->cap);
    return;
  }
  int done = 0;
  while (done < n) {
    if (rb->st_n == 0) rb->st_first = rb->total;
    const int take = std::min(n - done, kStageRows - rb->st_n);
    to_ring(rb, s + done * S, take * S, rb->st_s.data() + rb->st_n * S * es);
    to_ring(rb, s2 + done * S, take * S, rb->st_s2.data() + rb->st_n * S * es);
    to_ring(rb, r + done, take, rb->st_r.data() + rb->st_n * es);
    memcpy(rb->st_a.data() + rb->st_n * A, a + done * A, take * A * 4);
    for (int i = 0; i < take; ++i) rb->st_t[rb->st_n + i] = t[done + i] ? 1.f : 0.f;
    rb->st_n += take;
    rb->total += take;
    rb->count = std::min<int64_t>(rb->total, rb->cap);
    done += take;
    if (rb->st_n == kStageRows) replay_flush(rb);
  }
}
}  // extern "C++"

int ddpg_replay_add(ddpg_replay* rb, const float* s, const float* a, const float* r,
                    const uint8_t* t, const float* s2, int n) {
  return rguard(rb, [&] { replay_add_impl<float>(rb, s, a, r, t, s2, n); });
}

int ddpg_replay_add_f64(ddpg_replay* rb, const double* s, const float* a, const double* r,
                        const uint8_t* t, const double* s2, int n) {
  return rguard(rb, [&] { replay_add_impl<double>(rb, s, a, r, t, s2, n); });
}

int64_t ddpg_replay_size(ddpg_replay* rb) { return rb ? rb->count : 0; }
int64_t ddpg_replay_total_added(ddpg_replay* rb) { return rb ? rb->total : 0; }

int ddpg_replay_clear(ddpg_replay* rb) {
  return rguard(rb, [&] {
    HIP_TRY(hipStreamSynchronize(rb->stream));
    HIP_TRY(hipEventSynchronize(rb->written));
    rb->count = rb->total = 0;
    rb->st_n = 0;
  });
}

extern "C++" {
// ReplayBuffer.sample_batch to host arrays of type T (s, s2, r).  The rows are
// gathered on device in the ring's own precision (byte copies) and converted
// on the host: exact for a float64 ring read as float64 and for a fp32 ring.
template <class T>
static int sample_impl(ddpg_replay* rb, int B, T* s, float* a, T* r, uint8_t* t, T* s2,
                       int64_t* idx_out) {
  int got = 0;
  int rc = rguard(rb, [&] {
    if (B < 0) throw einval("negative batch");
    HIP_TRY(hipSetDevice(rb->device));
    replay_flush(rb);
    ring_join(rb);
    const int k = (int)std::min<int64_t>(B, rb->count);  // replay_buffer.py:36-39
    rb->tmp_idx.resize(std::max(1, k));
    if (rb->sampler.sample(rb->count, k, rb->tmp_idx.data()) != 0) throw einval("sample failed");
    got = k;
    if (idx_out) memcpy(idx_out, rb->tmp_idx.data(), k * sizeof(int64_t));
    if (k == 0) return;
    rb->tmp_slot.resize(k);
    for (int i = 0; i < k; ++i) rb->tmp_slot[i] = pos_to_slot(rb, rb->tmp_idx[i]);
    const size_t S = rb->S, A = rb->A, es = rb->es();
    if (rb->d_slots_cap < k) {
      if (rb->d_slots) HIP_TRY(hipFree(rb->d_slots));
      HIP_TRY(hipMalloc(&rb->d_slots, k * sizeof(int)));
      rb->d_slots_cap = k;
    }
    const size_t row_bytes = 2 * S * es + A * 4 + es + 4;
    const size_t need = (size_t)k * row_bytes;
    if (rb->d_tmp_cap < need) {
      if (rb->d_tmp) HIP_TRY(hipFree(rb->d_tmp));
      HIP_TRY(hipMalloc(&rb->d_tmp, need));
      rb->d_tmp_cap = need;
    }
    // output planes, each [k][row bytes]: s | s2 | a | r | t
    unsigned char* o_s = rb->d_tmp;
    unsigned char* o_s2 = o_s + k * S * es;
    unsigned char* o_a = o_s2 + k * S * es;
    unsigned char* o_r = o_a + k * A * 4;
    unsigned char* o_t = o_r + k * es;
    HIP_TRY(hipMemcpyAsync(rb->d_slots, rb->tmp_slot.data(), k * sizeof(int),
                           hipMemcpyHostToDevice, rb->stream));
    struct Plane {
      const unsigned char* src;
      unsigned char* dst;
      size_t bytes;
    } planes[5] = {{rb->ps(), o_s, S * es},
                   {rb->ps2(), o_s2, S * es},
                   {(const unsigned char*)rb->ra, o_a, A * 4},
                   {rb->pr(), o_r, es},
                   {(const unsigned char*)rb->rt, o_t, 4}};
    for (const Plane& pl : planes) {
      hipLaunchKernelGGL(gather_bytes_kernel, dim3(std::min(ceil_div(k, 4), 4096)), dim3(256), 0,
                         rb->stream, rb->d_slots, k, pl.src, pl.dst, (long long)pl.bytes);
      HIP_TRY(hipGetLastError());
    }
    std::vector<unsigned char> tmp(need);
    HIP_TRY(hipMemcpyAsync(tmp.data(), rb->d_tmp, need, hipMemcpyDeviceToHost, rb->stream));
    HIP_TRY(hipStreamSynchronize(rb->stream));
    auto conv = [&](const unsigned char* src, size_t n, T* dst) {
      if (!dst) return;
      if (rb->f64)
        for (size_t i = 0; i < n; ++i) dst[i] = (T)((const double*)src)[i];
      else
        for (size_t i = 0; i < n; ++i) dst[i] = (T)((const float*)src)[i];
    };
    const size_t off_s2 = k * S * es, off_a = 2 * off_s2, off_r = off_a + k * A * 4,
                 off_t = off_r + k * es;
    conv(tmp.data(), k * S, s);
    conv(tmp.data() + off_s2, k * S, s2);
    conv(tmp.data() + off_r, k, r);
    if (a) memcpy(a, tmp.data() + off_a, (size_t)k * A * 4);
    if (t)
      for (int i = 0; i < k; ++i) t[i] = ((const float*)(tmp.data() + off_t))[i] != 0.f;
  });
  return rc == DDPG_OK ? got : rc;
}
}  // extern "C++"

int ddpg_replay_sample_batch(ddpg_replay* rb, int B, float* s, float* a, float* r, uint8_t* t,
                             float* s2, int64_t* idx_out) {
  return sample_impl<float>(rb, B, s, a, r, t, s2, idx_out);
}

int ddpg_replay_sample_batch_f64(ddpg_replay* rb, int B, double* s, float* a, double* r,
                                 uint8_t* t, double* s2, int64_t* idx_out) {
  return sample_impl<double>(rb, B, s, a, r, t, s2, idx_out);
}

}  // extern "C"
