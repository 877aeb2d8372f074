// Native HIP runtime layer of the framework (C ABI, bound in textblaster_amd/ops/hiprt.py).
//
// The device path (pipeline/device.py, ops/kernels.py, ops/html.py) needs only a handful of
// runtime services: device selection, HBM and pinned host memory, streams, events, async copies
// and fills. They are provided here directly on the HIP runtime, so a single-GPU run never
// imports PyTorch (whose import alone costs ~1.5 s of process start-up, measured on the box:
// profiles/r2_e2e/). PyTorch remains the multi-rank layer (torch.distributed over RCCL).
//
// Memory: two caching allocators (device HBM, pinned host), best-fit over size-sorted free
// lists. A block is handed back to its cache only after the GPU work that used it completed
// (the Python side frees a batch's buffers after the batch's completion event), so reuse needs
// no stream bookkeeping. On hipErrorOutOfMemory the cache is flushed and the allocation
// retried once.
//
// Also here: k_scan_strided_i64, the inclusive prefix sum used for content-version offsets
// (C4 pass B, HTML decode) — one workgroup, each thread scanning a contiguous chunk.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Cache {
  std::mutex m;
  std::multimap<size_t, void*> free_blocks;     // size -> block
  std::unordered_map<void*, size_t> size_of;    // every live or cached block
  size_t cached = 0, in_use = 0, peak = 0;
};

constexpr int kMaxDevices = 64;
Cache g_dev[kMaxDevices];
Cache g_host;

size_t round_size(size_t n) {
  if (n == 0) n = 1;
  if (n <= (1u << 20)) return (n + 511) & ~size_t(511);
  return (n + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
}

void flush(Cache& c, bool host) {
  // caller holds c.m
  for (auto& kv : c.free_blocks) {
    if (host)
      (void)hipHostFree(kv.second);
    else
      (void)hipFree(kv.second);
    c.size_of.erase(kv.second);
  }
  c.free_blocks.clear();
  c.cached = 0;
}

int cache_alloc(Cache& c, bool host, void** out, size_t n) {
  const size_t sz = round_size(n);
  std::lock_guard<std::mutex> g(c.m);
  auto it = c.free_blocks.lower_bound(sz);
  // best fit, but never hand out a block more than twice (+2 MB) the request
  if (it != c.free_blocks.end() && it->first <= 2 * sz + (2u << 20)) {
    *out = it->second;
    c.cached -= it->first;
    c.in_use += it->first;
    if (c.in_use > c.peak) c.peak = c.in_use;
    c.free_blocks.erase(it);
    return 0;
  }
  void* p = nullptr;
  hipError_t e = host ? hipHostMalloc(&p, sz, hipHostMallocDefault) : hipMalloc(&p, sz);
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
    (void)hipGetLastError();
    flush(c, host);
    e = host ? hipHostMalloc(&p, sz, hipHostMallocDefault) : hipMalloc(&p, sz);
  }
  if (e != hipSuccess) return (int)e;
  c.size_of[p] = sz;
  c.in_use += sz;
  if (c.in_use > c.peak) c.peak = c.in_use;
  *out = p;
  return 0;
}

int cache_release(Cache& c, void* p) {
  if (!p) return 0;
  std::lock_guard<std::mutex> g(c.m);
  auto it = c.size_of.find(p);
  if (it == c.size_of.end()) return (int)hipErrorInvalidValue;
  c.free_blocks.emplace(it->second, p);
  c.cached += it->second;
  c.in_use -= it->second;
  return 0;
}

Cache* dev_cache() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) return nullptr;
  return &g_dev[d];
}

// inclusive prefix sum of src[i * stride], i < n -> out[i]; one workgroup of 1024 threads,
// thread t owns the contiguous chunk [t*chunk, (t+1)*chunk)
constexpr int kScanThreads = 1024;

__global__ __launch_bounds__(kScanThreads) void k_scan_strided_i64(const int64_t* __restrict__ src, int64_t stride,
                                                                    int64_t n, int64_t* __restrict__ out) {
  __shared__ int64_t sums[kScanThreads];
  const int t = threadIdx.x;
  const int64_t chunk = (n + kScanThreads - 1) / kScanThreads;
  const int64_t b = t * chunk;
  const int64_t e = b + chunk < n ? b + chunk : n;
  int64_t s = 0;
  for (int64_t i = b; i < e; ++i) s += src[i * stride];
  sums[t] = s;
  __syncthreads();
  // Hillis-Steele over the 1024 chunk sums
  for (int d = 1; d < kScanThreads; d <<= 1) {
    const int64_t v = t >= d ? sums[t - d] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int64_t run = t ? sums[t - 1] : 0;
  for (int64_t i = b; i < e; ++i) {
    run += src[i * stride];
    out[i] = run;
  }
}

}  // namespace

extern "C" {

int tbrt_device_count(int* n) { return (int)hipGetDeviceCount(n); }
int tbrt_set_device(int d) { return (int)hipSetDevice(d); }
int tbrt_get_device(int* d) { return (int)hipGetDevice(d); }
int tbrt_device_sync() { return (int)hipDeviceSynchronize(); }
int tbrt_mem_info(size_t* free_b, size_t* total_b) { return (int)hipMemGetInfo(free_b, total_b); }

int tbrt_malloc(void** p, size_t n) {
  Cache* c = dev_cache();
  if (!c) return (int)hipErrorInvalidDevice;
  return cache_alloc(*c, false, p, n);
}

int tbrt_free(void* p) {
  // blocks are tagged by address: look the block up in every device cache (few devices)
  for (int d = 0; d < kMaxDevices; ++d) {
    Cache& c = g_dev[d];
    std::lock_guard<std::mutex> g(c.m);
    auto it = c.size_of.find(p);
    if (it == c.size_of.end()) continue;
    c.free_blocks.emplace(it->second, p);
    c.cached += it->second;
    c.in_use -= it->second;
    return 0;
  }
  return (int)hipErrorInvalidValue;
}

int tbrt_host_alloc(void** p, size_t n) { return cache_alloc(g_host, true, p, n); }
int tbrt_host_free(void* p) { return cache_release(g_host, p); }

int tbrt_empty_cache() {
  for (int d = 0; d < kMaxDevices; ++d) {
    std::lock_guard<std::mutex> g(g_dev[d].m);
    if (!g_dev[d].free_blocks.empty()) flush(g_dev[d], false);
  }
  std::lock_guard<std::mutex> g(g_host.m);
  flush(g_host, true);
  return 0;
}

// stats[0..5] = device in_use, cached, peak, host in_use, cached, peak (current device)
int tbrt_cache_stats(size_t* stats) {
  Cache* c = dev_cache();
  if (!c) return (int)hipErrorInvalidDevice;
  {
    std::lock_guard<std::mutex> g(c->m);
    stats[0] = c->in_use;
    stats[1] = c->cached;
    stats[2] = c->peak;
  }
  std::lock_guard<std::mutex> g(g_host.m);
  stats[3] = g_host.in_use;
  stats[4] = g_host.cached;
  stats[5] = g_host.peak;
  return 0;
}

int tbrt_stream_create(hipStream_t* s, int priority) {
  // non-blocking: no implicit ordering against the legacy null stream
  return (int)hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority);
}
int tbrt_stream_destroy(hipStream_t s) { return (int)hipStreamDestroy(s); }
int tbrt_stream_sync(hipStream_t s) { return (int)hipStreamSynchronize(s); }
int tbrt_stream_priority_range(int* lo, int* hi) { return (int)hipDeviceGetStreamPriorityRange(lo, hi); }

int tbrt_event_create(hipEvent_t* e, int timing) {
  return (int)hipEventCreateWithFlags(e, timing ? hipEventDefault : hipEventDisableTiming);
}
int tbrt_event_destroy(hipEvent_t e) { return (int)hipEventDestroy(e); }
int tbrt_event_record(hipEvent_t e, hipStream_t s) { return (int)hipEventRecord(e, s); }
int tbrt_event_sync(hipEvent_t e) { return (int)hipEventSynchronize(e); }
// 0 = complete, 1 = pending, otherwise an error code + 2
int tbrt_event_query(hipEvent_t e) {
  const hipError_t r = hipEventQuery(e);
  if (r == hipSuccess) return 0;
  if (r == hipErrorNotReady) return 1;
  return (int)r + 2;
}
int tbrt_event_elapsed(float* ms, hipEvent_t a, hipEvent_t b) { return (int)hipEventElapsedTime(ms, a, b); }
int tbrt_stream_wait_event(hipStream_t s, hipEvent_t e) { return (int)hipStreamWaitEvent(s, e, 0); }

int tbrt_memcpy_h2d(void* dst, const void* src, size_t n, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
}
int tbrt_memcpy_d2h(void* dst, const void* src, size_t n, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
}
int tbrt_memcpy_d2d(void* dst, const void* src, size_t n, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s);
}
int tbrt_memset(void* p, int v, size_t n, hipStream_t s) { return (int)hipMemsetAsync(p, v, n, s); }

int tb_scan_strided_i64(hipStream_t stream, const int64_t* src, int64_t stride, int64_t n, int64_t* out) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_scan_strided_i64, dim3(1), dim3(kScanThreads), 0, stream, src, stride, n, out);
  return (int)hipGetLastError();
}

}  // extern "C"
