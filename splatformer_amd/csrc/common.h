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
// single-pass int32 scan (common.hip) on a look-back area (see there); lookback_state: the library-owned area of
// a (device, stream) with room for `words` tile words, plus a fresh tag for one scan on it
int lookback_state(hipStream_t st, long long words, unsigned** ticket, unsigned long long** flags, unsigned* tag);
long long lookback_scan_words(long long n);
void lookback_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, unsigned* ticket,
                       unsigned long long* flags, unsigned tag, int32_t* total, hipStream_t st);

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

// fp32 -> three bf16 terms by round-to-nearest (v_cvt_pk_bf16_f32): x = t0 + t1 + t2 + r with
// |t1| <= 2^-8 |x|, |t2| <= 2^-16 |x|, |r| <= 2^-24 |x| (each residual x - t0, (x - t0) - t1 is exact in fp32);
// bf16 keeps fp32's exponent range, so no scaling and no overflow cases.  The MFMA paths that run fp32
// products as the six leading term products (t0t0, t0t1, t1t0, t0t2, t1t1, t2t0) on bf16 MFMA with fp32
// accumulation (GEMM, window attention) are as accurate as fp32 arithmetic.
typedef __bf16 sfx_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const sfx_bf16x2 v = __builtin_convertvector((float __attribute__((ext_vector_type(2)))){a, b}, sfx_bf16x2);
  return __builtin_bit_cast(unsigned, v);
}
// 4 elements -> 3 terms x 4 packed bf16
__device__ __forceinline__ void split3(float4 v, uint2 (&t)[3]) {
  unsigned u0 = pk_bf16(v.x, v.y), u1 = pk_bf16(v.z, v.w);
  t[0] = make_uint2(u0, u1);
  float r0 = v.x - bf_lo(u0), r1 = v.y - bf_hi(u0), r2 = v.z - bf_lo(u1), r3 = v.w - bf_hi(u1);
  u0 = pk_bf16(r0, r1);
  u1 = pk_bf16(r2, r3);
  t[1] = make_uint2(u0, u1);
  r0 -= bf_lo(u0);
  r1 -= bf_hi(u0);
  r2 -= bf_lo(u1);
  r3 -= bf_hi(u1);
  t[2] = make_uint2(pk_bf16(r0, r1), pk_bf16(r2, r3));
}

// fp32 -> two fp16 terms of the scaled value (fp16x2 GEMM operands): x*s = h + l + r with h = fp16(x*s),
// l = fp16(x*s - h) (the residual x*s - h is exact in fp32), |r| <= 2^-22 |x*s|.  `s` is a power of two that
// puts the operand's largest magnitude in [2^14, 2^15), so no term overflows; elements far below the maximum
// lose bits of l only below 2^-24 of the maximum (fp16 subnormals).  h*h + h*l + l*h on fp16 MFMA with fp32
// accumulation has the error of fp32 arithmetic (dropped l*l <= 2^-22).
typedef _Float16 sfx_f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_f16(float a, float b) {
  const sfx_f16x2 v = __builtin_convertvector((float __attribute__((ext_vector_type(2)))){a, b}, sfx_f16x2);
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ void split2h(float4 v, float s, uint2 (&t)[2]) {
  const float x0 = v.x * s, x1 = v.y * s, x2 = v.z * s, x3 = v.w * s;
  const unsigned u0 = pk_f16(x0, x1), u1 = pk_f16(x2, x3);
  t[0] = make_uint2(u0, u1);
  const sfx_f16x2 h0 = __builtin_bit_cast(sfx_f16x2, u0), h1 = __builtin_bit_cast(sfx_f16x2, u1);
  t[1] = make_uint2(pk_f16(x0 - (float)h0.x, x1 - (float)h0.y), pk_f16(x2 - (float)h1.x, x3 - (float)h1.y));
}

// amax slots (fp16x2 GEMM operand scales): 64 u64 sub-slots holding (tag << 32 | bits of a non-negative float),
// written with atomicMax (larger tags supersede older contents), read as the max over the sub-slots that carry
// the expected tag.  Every lane of the calling wave returns the same value.
constexpr int kAmaxSub = 64;
__device__ __forceinline__ float read_amax(const unsigned long long* slot, unsigned tag) {
  const unsigned long long v = slot[__lane_id()];
  float m = ((unsigned)(v >> 32) == tag) ? __builtin_bit_cast(float, (unsigned)(v & 0xffffffffu)) : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, m)));
}
// workgroup-wide max of `m` (every thread calls it), one atomic into sub-slot blockIdx % 64
__device__ __forceinline__ void publish_amax(float m, unsigned long long* slot, unsigned tag, float* lds_waves) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int nw = (blockDim.x * blockDim.y + 63) / 64, w = (threadIdx.y * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) lds_waves[w] = m;
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r = fmaxf(r, lds_waves[i]);
    atomicMax(slot + (blockIdx.x + blockIdx.y * gridDim.x) % kAmaxSub,
              ((unsigned long long)tag << 32) | __builtin_bit_cast(unsigned, r));
  }
}

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
// Sum over the 64 lanes, result uniform (every lane): DPP butterflies inside each 16-lane row
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror) + the four row sums read back as scalars.
// No LDS traffic, unlike __shfl_xor (ds_bpermute).  bound_ctrl set (every lane of these patterns reads a
// valid lane, so it changes nothing) lets the compiler fold the move into v_add_f32_dpp.
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
  int t;
  switch (ctrl_sel) {
    case 0: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true); break;   // quad [1,0,3,2]
    case 1: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true); break;   // quad [2,3,0,1]
    case 2: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true); break;  // row_half_mirror
    default: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, true); break; // row_mirror
  }
  return v + __int_as_float(t);
}
// v of the lane the DPP control selects (quad_perm / row_ror / mirror patterns: every lane reads a valid lane)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = dpp_add(v, 0);
  v = dpp_add(v, 1);
  v = dpp_add(v, 2);
  v = dpp_add(v, 3);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- decoupled look-back (single-pass scan, one-sweep radix passes) ----------------------------------------
// A tile publishes one 8-byte status word per scanned quantity: tag (24 bits: which launch of the workspace it
// belongs to; a zeroed workspace holds tag 0 = "nothing yet") | status (aggregate / inclusive prefix) | 32-bit
// value.  The word is the whole hand-off (a data-tagged granule: written by ONE agent-scope store, `global_store
// ... sc1`, polled by agent-scope loads, `global_load ... sc1` -- MI355X_MICROARCH.md, Workgroup dispatch,
// "Valid forms"), so no fence orders anything else.  Tiles are numbered by a returning atomic ticket at
// workgroup start, so a tile only ever waits on tiles that are already running: no dispatch-order assumption.
constexpr unsigned kLbAgg = 1u, kLbPrefix = 2u;
__device__ __forceinline__ unsigned long long lb_word(unsigned tag, unsigned status, int value) {
  return ((unsigned long long)tag << 34) | ((unsigned long long)status << 32) | (unsigned)value;
}
__device__ __forceinline__ void lb_store(unsigned long long* p, unsigned long long w) {
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned lb_tag(unsigned long long w) { return (unsigned)(w >> 34); }
__device__ __forceinline__ unsigned lb_status(unsigned long long w) { return (unsigned)(w >> 32) & 3u; }
__device__ __forceinline__ int lb_value(unsigned long long w) { return (int)(unsigned)w; }
// Exclusive prefix of tile `tile` by a whole wave (uniform call): lanes read 64 predecessors at once, nearest first,
// adding aggregates until an inclusive prefix; spins (s_sleep) on words that do not carry `tag` yet.
// Every wait is bounded (kLbSpinCap polls, far above any real wait), so a broken hand-off cannot hang the GPU; a
// wait that reaches the cap goes on with the stale word and counts itself in `*timeouts` (the look-back area's
// header word, read by sfx_lookback_timeouts), so a wrong prefix is never silent.
constexpr int kLbSpinCap = 1 << 22;
__device__ __forceinline__ int lb_lookback_wave(const unsigned long long* flags, int tile, unsigned tag,
                                                unsigned* timeouts) {
  const int lane = __lane_id();
  int excl = 0;
  int j = tile - 1;
  int spins = 0;
  bool counted = false;
  while (j >= 0) {
    const int idx = j - lane;
    unsigned st = kLbPrefix;
    int val = 0;
    if (idx >= 0) {
      const unsigned long long w = lb_load(flags + idx);
      st = lb_tag(w) == tag ? lb_status(w) : 0u;
      val = lb_value(w);
    }
    const unsigned long long pre = __ballot(st == kLbPrefix);
    // nearest predecessor with a prefix (idx < 0 counts as one); none in this window: all 64 are aggregates
    const int stop = pre ? __ffsll((long long)pre) - 1 : 63;
    const unsigned long long need = (stop == 63) ? ~0ull : ((2ull << stop) - 1ull);
    if (__ballot(st == 0u) & need) {  // a needed predecessor has not published yet
      if (++spins < kLbSpinCap) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if (!counted && lane == 0) atomicAdd(timeouts, 1u);  // giving up: the prefix will be wrong, say so
      counted = true;
    }
    int v = (lane <= stop) ? val : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (pre) break;
    j -= 64;
  }
  return excl;
}

}  // namespace sfx

#define SFX_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::sfx::set_error(__VA_ARGS__);        \
      return SFX_ERR_INVALID;               \
    }                                       \
  } while (0)
