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
// (C4 pass B, HTML decode, K16 output compaction) — tile partials, then per-tile scans.
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

// Inclusive prefix sum of src[i * stride], i < n -> out[i], over the whole chip: k_scan_partials
// reduces each 2048-element tile (256 threads x 8 consecutive elements) to one partial, then
// k_scan_tiles gives every tile the sum of the partials before it (at most a few hundred, read by
// the whole workgroup) and scans the tile: thread-serial over its 8 elements, DPP-free wave scan of
// the thread totals with shuffles, and a 4-entry cross-wave pass in LDS. A 262,144-element scan is
// 128 workgroups per kernel instead of one 1024-thread workgroup walking everything.
constexpr int kScanThreads = 256;

std::mutex g_scan_mu;
std::map<std::pair<int, hipStream_t>, std::pair<int64_t*, int64_t>> g_scan_bufs;

int64_t* scan_partials_for(hipStream_t stream, int64_t n) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(g_scan_mu);
  auto& e = g_scan_bufs[{d, stream}];
  if (e.second < n) {
    if (e.first) (void)hipFree(e.first);
    e.first = nullptr;
    e.second = 0;
    const int64_t cap = n < 1024 ? 1024 : 2 * n;
    if (hipMalloc((void**)&e.first, (size_t)cap * sizeof(int64_t)) != hipSuccess) return nullptr;
    e.second = cap;
  }
  return e.first;
}
constexpr int kScanPer = 8;
constexpr int64_t kScanTile = (int64_t)kScanThreads * kScanPer;

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_partials(const int64_t* __restrict__ src, int64_t stride,
                                                                int64_t n, int64_t* __restrict__ partials) {
  __shared__ int64_t ws[kScanThreads / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = base + (int64_t)k * kScanThreads + t;  // coalesced for the reduction
    if (i < n) s += src[i * stride];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (lane == 0) ws[w] = s;
  __syncthreads();
  if (t == 0) {
    int64_t tot = 0;
    for (int k = 0; k < kScanThreads / 64; ++k) tot += ws[k];
    partials[blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(const int64_t* __restrict__ src, int64_t stride,
                                                             int64_t n, const int64_t* __restrict__ partials,
                                                             int64_t* __restrict__ out) {
  __shared__ int64_t ws[kScanThreads / 64];
  __shared__ int64_t tile_base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // sum of the partials of the tiles before this one
  int64_t pre = 0;
  for (int64_t k = t; k < (int64_t)blockIdx.x; k += kScanThreads) pre += partials[k];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d, 64);
  if (lane == 0) ws[w] = pre;
  __syncthreads();
  if (t == 0) {
    int64_t tot = 0;
    for (int k = 0; k < kScanThreads / 64; ++k) tot += ws[k];
    tile_base = tot;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * kScanTile + (int64_t)t * kScanPer;
  int64_t v[kScanPer];
  int64_t run = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = b0 + k;
    run += i < n ? src[i * stride] : 0;
    v[k] = run;
  }
  const int64_t incl = wave_incl_scan(run, lane);
  __syncthreads();  // ws reused
  if (lane == 63) ws[w] = incl;
  __syncthreads();
  int64_t off = tile_base + incl - run;
  for (int k = 0; k < w; ++k) off += ws[k];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = b0 + k;
    if (i < n) out[i] = off + v[k];
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

// flags: bit 0 = timing, bit 1 = blocking sync (the waiting host thread sleeps until the event
// signals instead of spinning a core: the batch pipeline waits ~20 ms per step on the device)
int tbrt_event_create(hipEvent_t* e, int flags) {
  unsigned f = (flags & 1) ? hipEventDefault : hipEventDisableTiming;
  if (flags & 2) f |= hipEventBlockingSync;
  return (int)hipEventCreateWithFlags(e, f);
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
  const int64_t tiles = (n + kScanTile - 1) / kScanTile;
  int64_t* partials = nullptr;
  if (tiles > 1) {
    // one partials buffer per (device, stream): scans on a stream run in order, so it is never
    // shared by two scans in flight; it only grows (hipFree synchronises before the old one goes)
    partials = scan_partials_for(stream, tiles);
    if (!partials) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL(k_scan_partials, dim3((uint32_t)tiles), dim3(kScanThreads), 0, stream, src, stride, n, partials);
  }
  hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)tiles), dim3(kScanThreads), 0, stream, src, stride, n, partials, out);
  return (int)hipGetLastError();
}

}  // extern "C"
