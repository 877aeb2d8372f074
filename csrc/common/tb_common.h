// Shared host/device definitions for textblaster_amd native code.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TB_HD __host__ __device__ __forceinline__
#define TB_DEV __device__ __forceinline__
#else
#define TB_HD inline
#define TB_DEV inline
#endif

namespace tb {

// Maximum n for the n-gram filters whose results are carried in fixed-size stat records.
constexpr int kMaxN = 32;

}  // namespace tb
