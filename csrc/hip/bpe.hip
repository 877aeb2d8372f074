// TokenCounter on the device (csrc/common/bpe.h): token counts of the kept outputs of K16.
//
// One wave per document (grid-stride over the documents). After k_compact the kept documents'
// final contents sit contiguously at the front of the output buffer, in document order; their
// number is the last entry of the kept-count scan, read here on the device, so counting follows
// compaction on the same stream with no host round trip. Each lane takes a 1/64 byte range of the
// document, finds the first pre-token start in it from the local boundary rules
// (bpe_first_start), and tokenizes + merges the pre-tokens that start in its range; the counts
// are summed across the wave. A lane's merge arrays live in LDS, interleaved by lane (element i
// of lane t at i * 64 + t: consecutive lanes, consecutive banks), 32 KB per 64-lane workgroup.
// A pre-token over those 64-byte arrays marks the document kBpeLong; k_bpe_long then recounts it
// with one wave per long pre-token (merge arrays of kBpeMaxLong entries, the minimum search spread
// over the wave).
#include <hip/hip_runtime.h>

#include "../common/bpe.h"

using namespace tb;

namespace {

constexpr int kBpeLanes = 64;
constexpr int kBpeMinChunk = 16;  // bytes per lane at least (short documents use fewer lanes)
constexpr int kBpeGrid = 8192;

__global__ __launch_bounds__(kBpeLanes) void k_bpe_count(DevBpe T, const uint8_t* __restrict__ text,
                                                         const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ n_dev, int32_t n_max,
                                                         int32_t* __restrict__ counts) {
  __shared__ uint32_t cs[kBpeMaxWord * kBpeLanes];
  __shared__ uint32_t rs[kBpeMaxWord * kBpeLanes];
  const int t = threadIdx.x;
  int64_t n = n_max;
  if (n_dev != nullptr) n = min(n, *n_dev);
  for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t s = off[k];
    const int64_t len = off[k + 1] - s;
    const uint8_t* b = text + s;
    const int64_t chunk = max((int64_t)kBpeMinChunk, (len + kBpeLanes - 1) / kBpeLanes);
    const int64_t s0 = (int64_t)t * chunk;
    long long cnt = 0;
    int bad = 0, lng = 0;
    if (s0 < len) {
      const int64_t s1 = min(len, s0 + chunk);
      if (T.n_added && bpe_has_added(T, b, len, s0, s1)) {
        bad = 1;
      } else {
        const int64_t x = bpe_count_range<true>(T, b, len, s0, s1, BpeArr{cs + t, kBpeLanes},
                                                BpeArr{rs + t, kBpeLanes}, [&](int64_t, int64_t) -> int64_t {
                                                  lng = 1;
                                                  return 0;
                                                });
        if (x < 0) bad = 1;
        else cnt = x;
      }
    }
    const bool any_bad = __ballot(bad) != 0, any_long = __ballot(lng) != 0;
    for (int o = kBpeLanes / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kBpeLanes);
    if (t == 0) {
      const long long tot = cnt + T.post_add;
      // (long pre-tokens: the tokens of the others travel in the count, k_bpe_long adds theirs)
      counts[k] = (any_bad || tot > 0x7FFFFFFF) ? kBpeHost : any_long ? (int32_t)(kBpeLong - tot) : (int32_t)tot;
    }
  }
}

constexpr int kBpeLongList = 32;  // long pre-tokens of one document counted on the device

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(x >> 32), o) << 32) | (uint32_t)__shfl_xor((int)x, o);
    x = y < x ? y : x;
  }
  return x;
}

// bpe_word_long (csrc/common/bpe.h) by one wave: the same linked-list merges, the search for the
// leftmost lowest-rank pair spread over the lanes; lane 0 applies each merge
__device__ int bpe_word_long_wave(const DevBpe& T, const uint8_t* w, int L, uint32_t* c, uint64_t* v, int16_t* nx,
                                  int16_t* pv, int lane) {
  if (L <= 1) return L;
  for (int i = lane; i < L; i += 64) {
    c[i] = T.byte_id[w[i]];
    nx[i] = (int16_t)(i + 1);
    pv[i] = (int16_t)(i - 1);
  }
  __syncthreads();
  for (int i = lane; i < L; i += 64) v[i] = i + 1 < L ? bpe_lookup(T, c[i], c[i + 1]) : ~0ull;
  __syncthreads();
  int m = L;
  while (m > 1) {
    uint64_t best = ~0ull;
    for (int i = lane; i < L; i += 64) {
      const uint64_t r = v[i] >> 32;
      if (r != kBpeNoRank) {
        const uint64_t key = (r << 32) | (uint32_t)i;  // rank, then position: the leftmost
        best = key < best ? key : best;
      }
    }
    best = wave_min_u64(best);
    if (best == ~0ull) break;
    if (lane == 0) {
      const int bi = (int)(uint32_t)best, j = nx[bi];
      c[bi] = (uint32_t)v[bi];
      nx[bi] = nx[j];
      if (nx[j] < L) pv[nx[j]] = (int16_t)bi;
      v[j] = ~0ull;
      v[bi] = nx[bi] < L ? bpe_lookup(T, c[bi], c[nx[bi]]) : ~0ull;
      if (pv[bi] >= 0) v[pv[bi]] = bpe_lookup(T, c[pv[bi]], c[bi]);
    }
    --m;
    __syncthreads();
  }
  return m;
}

// Documents k_bpe_count marked (count <= kBpeLong): the lanes delimit their ranges' pre-tokens
// again without merging the short ones (their tokens are in the mark), collect the long ones (up
// to kBpeLongList per document) and the wave merges them one after another.
__global__ __launch_bounds__(kBpeLanes) void k_bpe_long(DevBpe T, const uint8_t* __restrict__ text,
                                                        const int64_t* __restrict__ off,
                                                        const int64_t* __restrict__ n_dev, int32_t n_max,
                                                        int32_t* __restrict__ counts) {
  __shared__ uint32_t lc[kBpeMaxLong];
  __shared__ uint64_t lv[kBpeMaxLong];
  __shared__ int16_t lnx[kBpeMaxLong];
  __shared__ int16_t lpv[kBpeMaxLong];
  __shared__ int64_t ls[kBpeLongList], le[kBpeLongList];
  __shared__ uint32_t nlong;
  const int t = threadIdx.x;
  int64_t n = n_max;
  if (n_dev != nullptr) n = min(n, *n_dev);
  for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
    const int32_t mark = counts[k];
    if (mark > kBpeLong) continue;  // (uniform: one wave per block)
    const int64_t s = off[k];
    const int64_t len = off[k + 1] - s;
    const uint8_t* b = text + s;
    const int64_t chunk = max((int64_t)kBpeMinChunk, (len + kBpeLanes - 1) / kBpeLanes);
    const int64_t s0 = (int64_t)t * chunk;
    if (t == 0) nlong = 0;
    __syncthreads();
    long long cnt = 0;
    int bad = 0;
    if (s0 < len) {
      const int64_t x = bpe_count_range<false>(T, b, len, s0, min(len, s0 + chunk), BpeArr{nullptr, 0},
                                               BpeArr{nullptr, 0}, [&](int64_t a, int64_t e) -> int64_t {
                                          if (e - a > kBpeMaxLong) return -1;
                                          const uint32_t q = atomicAdd(&nlong, 1u);
                                          if (q >= (uint32_t)kBpeLongList) return -1;
                                          ls[q] = a;
                                          le[q] = e;
                                          return 0;
                                        });
      if (x < 0) bad = 1;
    }
    bool any_bad = __ballot(bad) != 0;
    cnt = (long long)kBpeLong - mark;  // the short pre-tokens' tokens and the post-processor's
    __syncthreads();
    const uint32_t nl = nlong < (uint32_t)kBpeLongList ? nlong : (uint32_t)kBpeLongList;
    for (uint32_t q = 0; q < nl && !any_bad; ++q)
      cnt += bpe_word_long_wave(T, b + ls[q], (int)(le[q] - ls[q]), lc, lv, lnx, lpv, t);
    if (t == 0) counts[k] = (any_bad || cnt > 0x7FFFFFFF) ? kBpeHost : (int32_t)cnt;
    __syncthreads();
  }
}

}  // namespace

// counts[k] for documents k < min(*n_dev, n_max) (n_dev may be null): text + off[k] .. off[k + 1]
extern "C" int tb_bpe_count(hipStream_t stream, const DevBpe* T, const uint8_t* text, const int64_t* off,
                            const int64_t* n_dev, int32_t n_max, int32_t* counts) {
  if (n_max <= 0) return 0;
  if (T == nullptr || T->n_added < 0 || T->n_added > kBpeMaxAdded) return (int)hipErrorInvalidValue;
  const int grid = n_max < kBpeGrid ? n_max : kBpeGrid;
  hipLaunchKernelGGL(k_bpe_count, dim3(grid), dim3(kBpeLanes), 0, stream, *T, text, off, n_dev, n_max, counts);
  // the documents with pre-tokens over kBpeMaxWord bytes (grid-stride; the others are skipped)
  const int grid_long = n_max < kBpeGrid / 4 ? n_max : kBpeGrid / 4;
  hipLaunchKernelGGL(k_bpe_long, dim3(grid_long), dim3(kBpeLanes), 0, stream, *T, text, off, n_dev, n_max, counts);
  return (int)hipGetLastError();
}

extern "C" size_t tb_sizeof_bpe() { return sizeof(DevBpe); }
