// Shared helpers for the libsfx HIP kernels (gfx950 / CDNA4 only).
//
// Every extern "C" entry point of the library follows the same contract
// (include/sfx.h): caller-owned device buffers, an explicit hipStream_t passed
// as `void*`, `int` status (0 = ok, negative = error) and a thread-local error
// string readable through sfx_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

#define SFX_OK 0
#define SFX_ERR_INVALID -1
#define SFX_ERR_HIP -2
#define SFX_ERR_WORKSPACE -3

namespace sfx {

void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return SFX_ERR_HIP;
  }
  return SFX_OK;
}

inline unsigned ceil_div(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

// 64-lane wavefront helpers ------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace sfx

#define SFX_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::sfx::set_error(__VA_ARGS__);        \
      return SFX_ERR_INVALID;               \
    }                                       \
  } while (0)
