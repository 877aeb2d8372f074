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
    int bad = 0;
    if (s0 < len) {
      const int64_t s1 = min(len, s0 + chunk);
      if (T.n_added && bpe_has_added(T, b, len, s0, s1)) {
        bad = 1;
      } else {
        const int64_t x = bpe_count_range(T, b, len, s0, s1, BpeArr{cs + t, kBpeLanes}, BpeArr{rs + t, kBpeLanes});
        if (x < 0) bad = 1;
        else cnt = x;
      }
    }
    const bool any_bad = __ballot(bad) != 0;
    for (int o = kBpeLanes / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kBpeLanes);
    if (t == 0) {
      const long long tot = cnt + T.post_add;
      counts[k] = (any_bad || tot > 0x7FFFFFFF) ? kBpeHost : (int32_t)tot;
    }
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
  return (int)hipGetLastError();
}

extern "C" size_t tb_sizeof_bpe() { return sizeof(DevBpe); }
