// Test-only stand-in for the RCCL calls of csrc/dp.hip, for running N real
// ranks (processes) of the data-parallel step on ONE GPU (RCCL refuses two
// ranks on one device: "Duplicate GPU detected").  Linked into a variant of
// the library (tools/build_shm_variant.sh -> tools/shm/libddpg_shm.so, loaded
// with DDPG_LIB_PATH by tests/test_gpu_dp_shm.py); the product library links
// RCCL itself and never contains this file.
//
// Each collective is executed at the call, host-synchronously: wait for the
// stream, copy this rank's bytes into its slot of a /dev/shm segment, barrier,
// reduce / gather from every slot IN RANK ORDER (so every rank computes the
// same bits), copy the result back to the device, barrier.  Groups are no-ops
// (every rank issues the same calls in the same order, as RCCL requires).
// Stream capture cannot contain host copies: run the step eagerly
// (DDPG_GRAPH_COMM=0).  Only what dp.hip uses: sum over float32, all-gather of
// float32 / bfloat16.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <new>
#include <vector>

namespace {

constexpr size_t kSlotBytes = 64ull << 20;  // per rank: the largest single call
constexpr int kMaxRanks = 16;

struct Header {
  std::atomic<int> arrived;
  std::atomic<int> generation;
  std::atomic<int> attached;
};

struct ShmComm {
  int world = 0, rank = 0;
  size_t map_bytes = 0;
  char* base = nullptr;
  char name[96] = {0};
  Header* hdr() { return reinterpret_cast<Header*>(base); }
  char* slot(int r) { return base + 4096 + (size_t)r * kSlotBytes; }
};

// sense-free generation barrier over the shared header (bounded: a peer that
// died leaves the survivors with an error instead of a hang)
bool barrier(ShmComm* c) {
  Header* h = c->hdr();
  const int gen = h->generation.load(std::memory_order_acquire);
  if (h->arrived.fetch_add(1, std::memory_order_acq_rel) == c->world - 1) {
    h->arrived.store(0, std::memory_order_relaxed);
    h->generation.store(gen + 1, std::memory_order_release);
    return true;
  }
  const time_t t0 = time(nullptr);
  while (h->generation.load(std::memory_order_acquire) == gen) {
    if (time(nullptr) - t0 > 60) return false;
    usleep(2);
  }
  return true;
}

size_t elt_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclFloat32: return 4;
    case ncclBfloat16: return 2;
    default: return 0;
  }
}

ncclResult_t d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (hipStreamSynchronize(s) != hipSuccess) return ncclUnhandledCudaError;
  if (bytes && hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return ncclUnhandledCudaError;
  return ncclSuccess;
}
ncclResult_t h2d(void* dst, const void* src, size_t bytes) {
  if (bytes && hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
    return ncclUnhandledCudaError;
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id, 0, sizeof *id);
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  snprintf(id->internal, sizeof id->internal, "/ddpg_shm_%d_%ld_%ld", (int)getpid(),
           (long)ts.tv_sec, (long)ts.tv_nsec);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int world, ncclUniqueId id, int rank) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return ncclInvalidArgument;
  ShmComm* c = new (std::nothrow) ShmComm;
  if (!c) return ncclSystemError;
  c->world = world;
  c->rank = rank;
  snprintf(c->name, sizeof c->name, "%s", id.internal);
  c->map_bytes = 4096 + (size_t)world * kSlotBytes;
  int fd = shm_open(c->name, O_RDWR | O_CREAT, 0600);
  if (fd < 0) return ncclSystemError;
  if (ftruncate(fd, (off_t)c->map_bytes) != 0) {  // same size from every rank: idempotent
    close(fd);
    return ncclSystemError;
  }
  void* p = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return ncclSystemError;
  c->base = static_cast<char*>(p);
  // a fresh segment reads zero: arrived = generation = attached = 0
  Header* h = c->hdr();
  h->attached.fetch_add(1, std::memory_order_acq_rel);
  const time_t t0 = time(nullptr);
  while (h->attached.load(std::memory_order_acquire) < world) {
    if (time(nullptr) - t0 > 120) return ncclSystemError;
    usleep(100);
  }
  if (!barrier(c)) return ncclSystemError;
  if (rank == 0) shm_unlink(c->name);  // every rank has it mapped
  *out = reinterpret_cast<ncclComm_t>(c);
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  ShmComm* c = reinterpret_cast<ShmComm*>(comm);
  if (!c) return ncclSuccess;
  munmap(c->base, c->map_bytes);
  delete c;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  return r == ncclSuccess ? "success (shm stand-in)" : "shm stand-in error";
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t t,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t s) {
  ShmComm* c = reinterpret_cast<ShmComm*>(comm);
  if (t != ncclFloat32 || op != ncclSum || count * 4 > kSlotBytes) return ncclInvalidArgument;
  ncclResult_t r = d2h(c->slot(c->rank), send, count * 4, s);
  if (r != ncclSuccess) return r;
  if (!barrier(c)) return ncclSystemError;
  std::vector<float> sum(count);
  const float* s0 = reinterpret_cast<const float*>(c->slot(0));
  for (size_t i = 0; i < count; ++i) sum[i] = s0[i];
  for (int w = 1; w < c->world; ++w) {
    const float* sw = reinterpret_cast<const float*>(c->slot(w));
    for (size_t i = 0; i < count; ++i) sum[i] += sw[i];
  }
  if (!barrier(c)) return ncclSystemError;  // slots free for the next call
  return h2d(recv, sum.data(), count * 4);
}

ncclResult_t ncclReduceScatter(const void* send, void* recv, size_t recvcount, ncclDataType_t t,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t s) {
  ShmComm* c = reinterpret_cast<ShmComm*>(comm);
  const size_t n = recvcount * c->world;
  if (t != ncclFloat32 || op != ncclSum || n * 4 > kSlotBytes) return ncclInvalidArgument;
  ncclResult_t r = d2h(c->slot(c->rank), send, n * 4, s);
  if (r != ncclSuccess) return r;
  if (!barrier(c)) return ncclSystemError;
  std::vector<float> sum(recvcount);
  const size_t o = recvcount * c->rank;
  const float* s0 = reinterpret_cast<const float*>(c->slot(0)) + o;
  for (size_t i = 0; i < recvcount; ++i) sum[i] = s0[i];
  for (int w = 1; w < c->world; ++w) {
    const float* sw = reinterpret_cast<const float*>(c->slot(w)) + o;
    for (size_t i = 0; i < recvcount; ++i) sum[i] += sw[i];
  }
  if (!barrier(c)) return ncclSystemError;
  return h2d(recv, sum.data(), recvcount * 4);
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t sendcount, ncclDataType_t t,
                           ncclComm_t comm, hipStream_t s) {
  ShmComm* c = reinterpret_cast<ShmComm*>(comm);
  const size_t eb = elt_bytes(t), bytes = sendcount * eb;
  if (!eb || bytes > kSlotBytes) return ncclInvalidArgument;
  ncclResult_t r = d2h(c->slot(c->rank), send, bytes, s);
  if (r != ncclSuccess) return r;
  if (!barrier(c)) return ncclSystemError;
  std::vector<char> all(bytes * c->world);
  for (int w = 0; w < c->world; ++w) memcpy(all.data() + w * bytes, c->slot(w), bytes);
  if (!barrier(c)) return ncclSystemError;
  return h2d(recv, all.data(), all.size());
}

}  // extern "C"
