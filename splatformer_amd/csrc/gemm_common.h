// Shared declarations of the fp32-accurate GEMM kernels (gemm.hip): launch arguments, epilogue helpers and
// raw-buffer access.
#pragma once

#include <type_traits>

#include "common.h"

namespace sfxg {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 32;
// residency: persistent workgroups per CU for the four- and eight-wave tiles, LDS buffers of the eight-wave ones
#ifndef SFX_PERCU4
#define SFX_PERCU4 2
#endif
#ifndef SFX_PERCU8
#define SFX_PERCU8 1
#endif
#ifndef SFX_NBUF8
#define SFX_NBUF8 2
#endif
constexpr int kPerCu4 = SFX_PERCU4, kPerCu8 = SFX_PERCU8;
constexpr int LDS_STRIDE = BK + 4;
constexpr int THREADS = 256;
constexpr unsigned OOB = 0x7ffffff0u;        // byte offset past every descriptor extent
constexpr int RSRC_FLAGS = 0x00020000;       // gfx950 raw buffer, 32-bit data

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3 };

struct GemmArgs {
  int M, N, K;         // K = S * Kseg when gathering
  const float* A;
  long long lda;
  const int* gidx;     // gather index, row stride gstride, or null
  int S, Kseg, gstride;
  const float* W;      // [N, K] (row stride ldw)
  long long ldw;
  const float* bias;   // [N] or null
  const float* scale;  // [N] or null  (folded BatchNorm)
  const float* shift;  // [N] or null
  int act, act_ncols;  // act applies to columns < act_ncols
  const float* R;      // residual [*, ldr] or null
  long long ldr;
  const int* ridx;     // residual row index (by output row) or null
  float* Y;
  long long ldy;
  float* Ypre;         // optional copy of the pre-residual value
  long long ldypre;
  long long gA, gW, gB, gY;  // grouped GEMM (blockIdx.z): per-group element strides
  const int* out_rows;       // tile row -> output row (or null)
  // offset-major sparse conv ("pair mode"): blockIdx.x walks a flat tile list over up to 27 slices;
  // slice k gathers A rows pair_in[pair_off[k] ..] and atomically adds into rows pair_out[...] with the
  // weight slice W + k * slice_w_stride.
  int pair_mode;
  const int* pair_in;
  const int* pair_out;
  int slice_tile_off[28];
  int slice_pair_off[28];
  int num_slices;
  long long slice_w_stride;
  // backward-pass epilogue terms (applied after the activation): v *= rowscale[row] (drop-path masks),
  // v *= act'(dact_pre[row, col]) for cols < act_ncols (GELU / ReLU on the pre-activation, tanh on its output)
  const float* rowscale;
  int pre_before_act;  // Ypre receives the pre-activation value (training forward saves it for act')
  const float* dact_pre;
  long long ld_dact;
  int dact;
  // Stream-K: the tiles x K-slabs iteration space is split evenly over the workgroups; a tile cut by a range
  // boundary gets partial sums (atomic add into a zero-filled output; the k-slab-0 owner adds the linear
  // epilogue terms).  Only for linear epilogues (no activation, no pre-residual copy, no in-place residual).
  int sk;
  // operand precision (see gemm_kernel): 0 exact fp32 MFMA, 2 fp16x2, 3 bf16x3; 1 = the reference-precision mode
  // (sfx_set_precision(1), the class of the reference's fp16 autocast training, train.py:240): the leading fp16
  // term only -- operands rounded to fp16 after the per-row power-of-two scaling, one product per block, fp32
  // accumulation and outputs.  Chosen in dispatch.
  int split;
  // fp16x2 operand maxima, as "amax slots": 64 sub-slots of (tag << 32 | float bits) written with atomicMax
  // by the producer of the tensor (one sub-slot per producing workgroup); a reader takes the max over the
  // sub-slots carrying the expected tag, so slots are reused without clearing.  Upper bounds are enough
  // (a looser bound only lowers the scale).
  const unsigned long long* a_amax;
  const unsigned long long* w_amax;
  unsigned a_tag, w_tag;
  unsigned long long* y_amax;  // optional: max |Y| of this launch's outputs -> slot, tag y_tag
  unsigned y_tag;
  // pre-split W (sfx_weight_split): W's element layout in 4-byte units, every group
  // of 4 consecutive elements held as 4 fp16 h terms then 4 fp16 l terms of W[n, k] * 2^e_n; winv[n] = 2^-e_n.
  // Slices / groups use the same element offsets as W (slice_w_stride, gW); winv is grouped by gWinv.
  const float* Wsp;
  long long ldws;
  const float* winv;
  long long gWinv;
  long long slice_winv_stride;  // pair mode: winv offset per slice (row-sliced weights, e.g. the conv backward)
  int tuned, tuned_sk;  // measured tile configuration + 1 (0: cost model / table) and its Stream-K flag
  int pair_store;  // pair mode: store each pair's row at row `pair index` of Y instead of adding into pair_out
  // timing ablations only (SFX_GEMM_DEBUG, results wrong): bit 0 no MFMAs, 1 no operand loads (out-of-range
  // offsets), 2 no epilogue, 3 no LDS staging (split + writes)
  int dbg;
};

// fp16x2 row exponent: a row with maximum m is scaled by 2^e so that m * 2^e lies in [2^12, 2^13)
__device__ __forceinline__ int row_exp(float m) {
  int e = __builtin_amdgcn_frexp_expf(m);  // m in [2^(e-1), 2^e)
  e = 13 - e;
  return e > 126 ? 126 : (e < -126 ? -126 : e);
}

// erf GELU (torch approximate='none'), GELU(x) = x Phi(x), with Phi from ONE fitted exponent: the upper normal tail
// is erfc(t / sqrt 2) = 2^-h(t) with h(t) = t Q(t), Q a degree-7 polynomial (weighted least squares on [0, 5.65]
// against scipy's erfc in fp64, weights = the tail itself, so the fit is tight where it matters for Phi), t = |x|
// clamped to 5.65 (Phi(5.65) = 1 - 8e-9 rounds to 1).  Phi = 1 - tail / 2 (x >= 0) or tail / 2: max |Phi - Phi_exact|
// = 6.2e-8 over [-8, 8] in fp32 evaluation, the rounding level of Phi itself.  Branch-free and 16 VALU (one
// v_exp_f32) against ~25 for the two-range erf it replaced -- GELU is the fused MLP's VALU bottleneck
// (profiles/r04_mlp_gelu_variants.txt: the MLP ran 1.3-1.5x faster with GELU removed).
__device__ __forceinline__ float gelu_erf(float x) {
  const float t = fminf(fabsf(x), 5.65f);
  float q = 2.79405867e-06f;
  q = __builtin_fmaf(q, t, -3.89084234e-05f);
  q = __builtin_fmaf(q, t, 0.000184072458f);
  q = __builtin_fmaf(q, t, 0.000141672252f);
  q = __builtin_fmaf(q, t, -0.00706906663f);
  q = __builtin_fmaf(q, t, 0.0524996631f);
  q = __builtin_fmaf(q, t, 0.459207207f);
  q = __builtin_fmaf(q, t, 1.15110528f);
  const float half_tail = 0.5f * __builtin_amdgcn_exp2f(-(t * q));
  // below -5.65 the clamped tail would leave x * 4e-9, growing with |x|: exact GELU is 0 there (to below fp32's
  // rounding of the product), so the negative branch selects 0 (one v_cndmask)
  return x >= 0.f ? x * (1.f - half_tail) : (x < -5.65f ? 0.f : x * half_tail);
}
// d/dx of the erf GELU (torch GeluBackward, approximate='none').  Exact erff / expf, while the forward epilogues use
// the fitted gelu_erf above: the two differ by the fit's 6e-8 on Phi, far inside the training gradient bars
// (the backward's derivative is not the derivative of the fitted forward, by that margin)
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}
enum DAct { DACT_NONE = 0, DACT_GELU = 1, DACT_RELU = 2, DACT_TANH_OUT = 3 };
__device__ __forceinline__ float dact_grad(int dact, float pre) {
  if (dact == DACT_GELU) return gelu_erf_grad(pre);
  if (dact == DACT_RELU) return pre > 0.f ? 1.f : 0.f;
  return 1.f - pre * pre;  // DACT_TANH_OUT: pre holds tanh(z)
}

// descriptor from a pointer that is wave-uniform by construction; readfirstlane makes that provable to
// hipcc, which otherwise wraps every buffer op in a waterfall loop (cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* u = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, (int)OOB, RSRC_FLAGS);
}

// descriptor with an explicit extent (bytes): accesses at or past it are dropped / read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_ext(const void* p, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* u = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), RSRC_FLAGS);
}

__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const floatx4 v = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ int bload1i(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void bstore1(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

using sfx::split3;   // fp32 -> three bf16 terms (common.h)
using sfx::split2h;  // fp32 -> two fp16 terms of the scaled value (common.h)

enum Mode { MODE_DENSE = 0, MODE_GATHER1 = 1, MODE_GATHERS = 2, MODE_PAIR = 3 };

// CUs of the current device (cached per process)
inline int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// M-tiles of a launch: plain ceil(M / BM), or per-slice rounding in pair mode (fills slice_tile_off)
inline int tiles_m_of(GemmArgs& a, int BM) {
  if (!a.pair_mode) return (int)sfx::ceil_div(a.M, BM);
  int t = 0;
  for (int k = 0; k < a.num_slices; ++k) {
    a.slice_tile_off[k] = t;
    t += (a.slice_pair_off[k + 1] - a.slice_pair_off[k] + BM - 1) / BM;
  }
  a.slice_tile_off[a.num_slices] = t;
  return t;
}

// Launchers of gemm_kernel (gemm_kernel.h), one translation unit per operand mode and wave count
// (gemm_k<mode><4|8>.hip, compiled in parallel): cfg indexes gemm.hip's kCfgs (0-4 four-wave, 5-6 eight-wave).
void launch_m0_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m0_w8(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m1_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m1_w8(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m2_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m3_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);
void launch_m3_w8(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st);

}  // namespace sfxg
