// Row-wise LayerNorm kernels for the PTv3 Block (pre-norm, eps 1e-5,
// nn.LayerNorm semantics: biased variance, affine).  One wave per row, the
// row held in registers (C <= 512 -> 8 floats per lane), two-pass mean /
// centred variance.
//
// sfx_layernorm          : Y = LN(X)                          (Block.norm1/norm2)
// sfx_cpe_residual_ln    : X' = X + LN_cpe(T); H = LN1(X')    (Block.forward: cpe tail,
//                          shortcut add and norm1 fused; reference calflops.py:45-53)
#include "common.h"

namespace {

constexpr int MAXV = 8;  // C <= 512

__device__ __forceinline__ void ln_row(const float* v, int C, int lane, const float* __restrict__ g,
                                       const float* __restrict__ b, float eps, float* out) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) s += v[i];
  }
  s = sfx::wave_sum(s);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      const float d = v[i] - mean;
      q += d * d;
    }
  }
  q = sfx::wave_sum(q);
  const float rstd = 1.f / sqrtf(q / (float)C + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) out[i] = (v[i] - mean) * rstd * g[c] + b[c];
  }
}

__global__ void __launch_bounds__(256) layernorm_kernel(int M, int C, const float* __restrict__ X, long long ldx,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        float eps, float* __restrict__ Y, long long ldy) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  float v[MAXV], o[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? X[(long long)row * ldx + c] : 0.f;
  }
  ln_row(v, C, lane, g, b, eps, o);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) Y[(long long)row * ldy + c] = o[i];
  }
}

__global__ void __launch_bounds__(256) cpe_residual_ln_kernel(int M, int C, const float* __restrict__ T,
                                                              const float* __restrict__ X,
                                                              const float* __restrict__ g_cpe,
                                                              const float* __restrict__ b_cpe,
                                                              const float* __restrict__ g1,
                                                              const float* __restrict__ b1, float eps,
                                                              float* __restrict__ Xout, float* __restrict__ H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  float v[MAXV], o[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? T[(long long)row * C + c] : 0.f;
  }
  ln_row(v, C, lane, g_cpe, b_cpe, eps, o);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      v[i] = X[(long long)row * C + c] + o[i];
      Xout[(long long)row * C + c] = v[i];
    }
  }
  ln_row(v, C, lane, g1, b1, eps, o);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) H[(long long)row * C + c] = o[i];
  }
}


// ---- vectorised variants: a row is held by G lanes (float4 each, NV float4 per lane), G | 64, so one wave
// covers 64/G rows with 16-byte loads/stores.  C = 4 * G * NV in {64, 96, 128, 256, 512}.
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int G, int NV>
__device__ __forceinline__ void ln_row4(float4 (&v)[NV], const float* __restrict__ g, const float* __restrict__ b,
                                        float eps, int sub, float4 (&o)[NV]) {
  constexpr int C = 4 * G * NV;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = group_sum<G>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q += (a * a + bb * bb) + (c * c + d * d);
  }
  const float rstd = 1.f / sqrtf(group_sum<G>(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (sub + G * i);
    const float4 gg = *reinterpret_cast<const float4*>(g + c);
    const float4 bv = *reinterpret_cast<const float4*>(b + c);
    o[i] = make_float4((v[i].x - mean) * rstd * gg.x + bv.x, (v[i].y - mean) * rstd * gg.y + bv.y,
                       (v[i].z - mean) * rstd * gg.z + bv.z, (v[i].w - mean) * rstd * gg.w + bv.w);
  }
}

template <int G, int NV>
__global__ void __launch_bounds__(256) layernorm4_kernel(int M, const float* __restrict__ X, long long ldx,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, float* __restrict__ Y, long long ldy) {
  const int row = blockIdx.x * (256 / G) + threadIdx.x / G;
  const int sub = threadIdx.x % G;
  if (row >= M) return;
  float4 v[NV], o[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const float4*>(X + (long long)row * ldx + 4 * (sub + G * i));
  ln_row4<G, NV>(v, g, b, eps, sub, o);
#pragma unroll
  for (int i = 0; i < NV; ++i) *reinterpret_cast<float4*>(Y + (long long)row * ldy + 4 * (sub + G * i)) = o[i];
}

// t += the row's SubM pair partials (sfx_subm_conv_partials), offsets in ascending order: the conv output
// without float atomics, identical from run to run.  Absent pairs read through an out-of-range buffer offset (0).
template <int G, int NV>
__device__ __forceinline__ void add_pair_partials(float4 (&v)[NV], const float* __restrict__ P,
                                                  const int* __restrict__ pos, int row, int sub) {
  constexpr int C = 4 * G * NV;
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P), (short)0, 0x7ffffff0,
                                                                      0x00020000);
  if constexpr (G == 64 && NV == 1) {
    // one row per wave: the row's 27 pair positions are wave-uniform -- scalar loads (all first, so they batch),
    // then the 27 row loads back to back (absent offsets through an out-of-range offset: no branch, whose join
    // would make hipcc wait for every load before it)
    const int rowu = __builtin_amdgcn_readfirstlane(row);
    const int* pr = pos + 27ll * rowu;
    int q[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) q[k] = __builtin_amdgcn_readfirstlane(pr[k]);
    float4 a[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      const unsigned off = q[k] >= 0 ? ((unsigned)q[k] * (unsigned)C + 4u * (unsigned)sub) * 4u : 0x7ffffff0u;
      a[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0));
    }
#pragma unroll
    for (int k = 0; k < 27; ++k) v[0] = make_float4(v[0].x + a[k].x, v[0].y + a[k].y, v[0].z + a[k].z, v[0].w + a[k].w);
    return;
  }
  int q[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) q[k] = pos[27ll * row + k];
#pragma unroll
  for (int k = 0; k < 27; ++k) {  // (k = 13: the centre's row when the pair lists carry it, else -1: adds 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const unsigned off = q[k] >= 0 ? ((unsigned)q[k] * (unsigned)C + 4u * (unsigned)(sub + G * i)) * 4u : 0x7ffffff0u;
      const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0));
      v[i] = make_float4(v[i].x + a.x, v[i].y + a.y, v[i].z + a.z, v[i].w + a.w);
    }
  }
}

// The same sum from the compacted positions (sfx_subm_pair_lists pair_cpos [n][32]: the row's present pairs in
// ascending offset order, -1 after them, the count in element 31): the wave loops over ceil(max count / 8) groups of 8
// positions (two 16-byte index loads, 8 NV row loads, out-of-range past the row's count) instead of 27 position
// loads and 27 NV row loads of which ~90 % are out of range at 100k points; same order of additions.
template <int G, int NV>
__device__ __forceinline__ void add_pair_partials_c(float4 (&v)[NV], const float* __restrict__ P,
                                                    const int* __restrict__ cpos, int row, int sub) {
  constexpr int C = 4 * G * NV;
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P), (short)0, 0x7ffffff0,
                                                                      0x00020000);
  if constexpr (G == 64 && NV == 1) {  // one row per wave: scalar count and positions, loads for present pairs only
    const int* cu = cpos + 32ll * __builtin_amdgcn_readfirstlane(row);
    const int n = __builtin_amdgcn_readfirstlane(cu[31]);
    for (int j0 = 0; j0 < n; j0 += 8) {
      int q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = __builtin_amdgcn_readfirstlane(cu[j0 + u]);
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const unsigned off = j0 + u < n ? ((unsigned)q[u] * (unsigned)C + 4u * (unsigned)sub) * 4u : 0x7ffffff0u;
        a[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) v[0] = make_float4(v[0].x + a[u].x, v[0].y + a[u].y, v[0].z + a[u].z, v[0].w + a[u].w);
    }
    return;
  }
  const int* cr = cpos + 32ll * row;
  const int cnt = cr[31];
  int jmax = cnt;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) jmax = max(jmax, __shfl_xor(jmax, o, 64));
  jmax = __builtin_amdgcn_readfirstlane(jmax);
  for (int j0 = 0; j0 < jmax; j0 += 8) {
    const int4 qa = *reinterpret_cast<const int4*>(cr + j0), qb = *reinterpret_cast<const int4*>(cr + j0 + 4);
    const int q[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
    float4 a[8][NV];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const unsigned off =
            j0 + u < cnt ? ((unsigned)q[u] * (unsigned)C + 4u * (unsigned)(sub + G * i)) * 4u : 0x7ffffff0u;
        a[u][i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0));
      }
#pragma unroll
    for (int u = 0; u < 8; ++u)  // (past the count: + 0, as the [n][27] form adds for absent offsets)
#pragma unroll
      for (int i = 0; i < NV; ++i)
        v[i] = make_float4(v[i].x + a[u][i].x, v[i].y + a[u][i].y, v[i].z + a[u][i].z, v[i].w + a[u][i].w);
  }
}

// PAIRS: 0 T is the conv output, 1 add the pair partials named by pair_pos [n][27], 2 by pair_cpos [n][32]
template <int G, int NV, int PAIRS>
__global__ void __launch_bounds__(256) cpe_residual_ln4_kernel(int M, const float* __restrict__ T, long long ldt,
                                                               const float* __restrict__ X,
                                                               const float* __restrict__ g_cpe,
                                                               const float* __restrict__ b_cpe,
                                                               const float* __restrict__ g1,
                                                               const float* __restrict__ b1, float eps,
                                                               float* __restrict__ Xout, float* __restrict__ H,
                                                               const float* __restrict__ P,
                                                               const int* __restrict__ pos) {
  constexpr int C = 4 * G * NV;
  const int row = blockIdx.x * (256 / G) + threadIdx.x / G;
  const int sub = threadIdx.x % G;
  if (row >= M) return;
  const long long base = (long long)row * C;
  float4 v[NV], o[NV], x[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = *reinterpret_cast<const float4*>(T + (long long)row * ldt + 4 * (sub + G * i));
    x[i] = *reinterpret_cast<const float4*>(X + base + 4 * (sub + G * i));
  }
  if constexpr (PAIRS == 1) add_pair_partials<G, NV>(v, P, pos, row, sub);
  if constexpr (PAIRS == 2) add_pair_partials_c<G, NV>(v, P, pos, row, sub);
  ln_row4<G, NV>(v, g_cpe, b_cpe, eps, sub, o);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = make_float4(x[i].x + o[i].x, x[i].y + o[i].y, x[i].z + o[i].z, x[i].w + o[i].w);
    *reinterpret_cast<float4*>(Xout + base + 4 * (sub + G * i)) = v[i];
  }
  ln_row4<G, NV>(v, g1, b1, eps, sub, o);
#pragma unroll
  for (int i = 0; i < NV; ++i) *reinterpret_cast<float4*>(H + base + 4 * (sub + G * i)) = o[i];
}

// ---- pair-sum CPE LayerNorm + shortcut + norm1 + the qkv projection in one launch (eval Block, C <= 128) --------
// The Block's front half after its SubM conv (calflops.py:45-53 cpe tail, shortcut, norm1; :55 attn.qkv): per row
// t = T + sum_k partials (ascending k), x1 = X + LN_cpe(t) (written: the attention's residual), h = LN1(x1) -- kept
// on chip -- and qkv = h W^T + b (written, with max |qkv| published for the attention's fp16x2 scale).  h never
// reaches HBM and the qkv GEMM launch is gone.
// Mapping: wave w owns 32 consecutive rows.  Phase A (the LayerNorms, G lanes per row as cpe_residual_ln4_kernel,
// identical arithmetic) splits each h row into fp16x2 terms at the row's own power-of-two scale (max in
// [2^14, 2^15)) and stores them in the wave's LDS image [2 terms][32 rows][C fp16] (16-byte chunks XOR-swizzled by
// row: spread fragment reads).  Phase B: qkv^T[32 features][32 points] per chunk of 32 features on
// v_mfma_f32_32x32x16_f16 (h*h + h*l + l*h, fp32 accumulation): A = the pre-split W rows (sfx_weight_split, read
// from L2), B = the wave's h image (all k-steps held in registers across the 3C / 32 chunks); the epilogue unscales
// by the feature's and the point's scale, adds the bias and stores 16-byte row pieces.
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int G, int NV>
__global__ void __launch_bounds__(256) cpe_ln_qkv_kernel(int M, const float* __restrict__ T, long long ldt,
                                                         const float* __restrict__ P, const int* __restrict__ pos,
                                                         const float* __restrict__ X, const float* __restrict__ g_cpe,
                                                         const float* __restrict__ b_cpe,
                                                         const float* __restrict__ g1, const float* __restrict__ b1,
                                                         float eps, float* __restrict__ X1,
                                                         const uint4* __restrict__ wsp, const float* __restrict__ winv,
                                                         const float* __restrict__ bq, float* __restrict__ QKV,
                                                         unsigned long long* __restrict__ amax, unsigned tag) {
  constexpr int C = 4 * G * NV, N = 3 * C, NCHK = N / 32, KS = C / 16, RPP = 64 / G;
  constexpr int ROWB = 2 * C;  // bytes per image row and term
  static_assert(C % 64 == 0 || C == 96, "C");
  __shared__ __attribute__((aligned(16))) char himg[4][2][32 * ROWB];
  __shared__ float rsc[4][32];
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, sub = lane % G, grp = lane / G;
  const int r0 = blockIdx.x * 128 + 32 * wid;
  char* H0 = himg[wid][0];
  char* H1 = himg[wid][1];
  // 16-byte chunk c of row r at c ^ (r & SW): SW = 7 when a row holds a multiple of 8 chunks (C = 64, 128), 3 for
  // C = 96's 12 chunks (the XOR must stay inside the row)
  constexpr int SW = (C / 8) % 8 == 0 ? 7 : 3;
  auto hoff = [](int r, int c) -> int { return r * ROWB + ((c ^ (r & SW)) << 4); };

  // ---- phase A: LayerNorms (cpe_residual_ln4_kernel's arithmetic), h -> the wave's fp16x2 image ----
#pragma unroll 1
  for (int p = 0; p < 32 / RPP; ++p) {
    const int lr = p * RPP + grp;
    const int row = r0 + lr;
    float4 o[NV];
    if (row < M) {
      float4 v[NV], x[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        v[i] = *reinterpret_cast<const float4*>(T + (long long)row * ldt + 4 * (sub + G * i));
        x[i] = *reinterpret_cast<const float4*>(X + (long long)row * C + 4 * (sub + G * i));
      }
      add_pair_partials<G, NV>(v, P, pos, row, sub);
      ln_row4<G, NV>(v, g_cpe, b_cpe, eps, sub, o);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        v[i] = make_float4(x[i].x + o[i].x, x[i].y + o[i].y, x[i].z + o[i].z, x[i].w + o[i].w);
        *reinterpret_cast<float4*>(X1 + (long long)row * C + 4 * (sub + G * i)) = v[i];
      }
      ln_row4<G, NV>(v, g1, b1, eps, sub, o);
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) m = fmaxf(m, fmaxf(fmaxf(fabsf(o[i].x), fabsf(o[i].y)), fmaxf(fabsf(o[i].z), fabsf(o[i].w))));
    m = group_max<G>(m);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) {
      (void)frexpf(m, &e);
      e = 15 - e;
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    }
    const float sc = ldexpf(1.f, e);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c0 = 4 * (sub + G * i);  // channels c0 .. c0 + 3: half (c0 & 4) of 16-byte chunk c0 / 8
      uint2 t[2];
      sfx::split2h(o[i], sc, t);
      const int off = hoff(lr, c0 >> 3) + ((c0 & 4) << 1);
      *reinterpret_cast<uint2*>(H0 + off) = t[0];
      *reinterpret_cast<uint2*>(H1 + off) = t[1];
    }
    if (sub == 0) rsc[wid][lr] = ldexpf(1.f, -e);
  }
  __syncthreads();

  // ---- phase B: qkv^T chunks of 32 features for the wave's 32 points (lane = point) ----
  const int l32 = lane & 31, h = lane >> 5;
  const float ri = rsc[wid][l32];
  const int prow = r0 + l32;
  f16x8 bh[KS], bl[KS];
#pragma unroll
  for (int t = 0; t < KS; ++t) {
    const int off = hoff(l32, 2 * t + h);
    bh[t] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(H0 + off));
    bl[t] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(H1 + off));
  }
  float mx = 0.f;
#pragma unroll 1
  for (int ck = 0; ck < NCHK; ++ck) {
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const uint4* wr = wsp + (long long)(ck * 32 + l32) * (C / 4);
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const uint4 a = wr[4 * t + 2 * h], b = wr[4 * t + 2 * h + 1];  // k = 16 t + 8 h .. + 7 of feature row n
      const f16x8 wh = __builtin_bit_cast(f16x8, make_uint4(a.x, a.y, b.x, b.y));
      const f16x8 wl = __builtin_bit_cast(f16x8, make_uint4(a.z, a.w, b.z, b.w));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, bh[t], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, bl[t], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, bh[t], acc, 0, 0, 0);
    }
    if (prow < M) {
      float* dst = QKV + (long long)prow * N + ck * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n0 = ck * 32 + 8 * g + 4 * h;
        const float4 wi = *reinterpret_cast<const float4*>(winv + n0);
        const float4 bb = *reinterpret_cast<const float4*>(bq + n0);
        float4 y;
        y.x = acc[4 * g + 0] * (wi.x * ri) + bb.x;
        y.y = acc[4 * g + 1] * (wi.y * ri) + bb.y;
        y.z = acc[4 * g + 2] * (wi.z * ri) + bb.z;
        y.w = acc[4 * g + 3] * (wi.w * ri) + bb.w;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
        *reinterpret_cast<float4*>(dst + 8 * g + 4 * h) = y;
      }
    }
  }
  if (amax) sfx::publish_amax(mx, amax, tag, red);
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// |LN(x)_c| = |z_c gamma_c + beta_c| with |z_c| <= sqrt(C - 1) (biased variance, eps only shrinks z)
__global__ void __launch_bounds__(64) ln_amax_bound_kernel(int C, const float* __restrict__ g,
                                                            const float* __restrict__ b,
                                                            unsigned long long* __restrict__ slot, unsigned tag) {
  __shared__ float red[1];
  float mg = 0.f, mb = 0.f;  // one wave: both maxima are complete before the bound is formed
  for (int c = threadIdx.x; c < C; c += 64) {
    mg = fmaxf(mg, fabsf(g[c]));
    mb = fmaxf(mb, fabsf(b[c]));
  }
  mg = sfx::wave_max(mg);
  mb = sfx::wave_max(mb);
  const float bound = sqrtf((float)(C > 1 ? C - 1 : 1)) * mg * 1.0001f + mb;
  sfx::publish_amax(bound, slot, tag, red);
}

}  // namespace

extern "C" {

int sfx_ln_amax_bound(int C, const float* gamma, const float* beta, unsigned long long* slot, unsigned tag,
                      void* stream) {
  SFX_REQUIRE(C > 0 && gamma && beta && slot && tag != 0, "sfx_ln_amax_bound: bad arguments");
  ln_amax_bound_kernel<<<1, 64, 0, sfx::as_stream(stream)>>>(C, gamma, beta, slot, tag);
  return sfx::check_launch("sfx_ln_amax_bound");
}

int sfx_layernorm(int M, int C, const float* X, long long ldx, const float* gamma, const float* beta, float eps,
                  float* Y, long long ldy, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_layernorm: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(X && gamma && beta && Y, "sfx_layernorm: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const bool v4 = ldx % 4 == 0 && ldy % 4 == 0 && al16(X) && al16(Y) && al16(gamma) && al16(beta);
#define SFX_LN4(G, NV) layernorm4_kernel<G, NV><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, X, ldx, gamma, beta, eps, Y, ldy)
  if (v4 && C == 64) SFX_LN4(16, 1);
  else if (v4 && C == 96) SFX_LN4(8, 3);
  else if (v4 && C == 128) SFX_LN4(32, 1);
  else if (v4 && C == 256) SFX_LN4(64, 1);
  else if (v4 && C == 512) SFX_LN4(64, 2);
  else layernorm_kernel<<<sfx::ceil_div(M, 4), 256, 0, st>>>(M, C, X, ldx, gamma, beta, eps, Y, ldy);
#undef SFX_LN4
  return sfx::check_launch("sfx_layernorm");
}

int sfx_cpe_residual_ln(int M, int C, const float* T, const float* X, const float* gamma_cpe, const float* beta_cpe,
                        const float* gamma1, const float* beta1, float eps, float* X_out, float* H, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_cpe_residual_ln: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(T && X && gamma_cpe && beta_cpe && gamma1 && beta1 && X_out && H, "sfx_cpe_residual_ln: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const bool v4 = al16(T) && al16(X) && al16(X_out) && al16(H) && al16(gamma_cpe) && al16(beta_cpe) && al16(gamma1) &&
                  al16(beta1);
#define SFX_CPE4(G, NV)                                                                                         \
  cpe_residual_ln4_kernel<G, NV, 0><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, T, C, X, gamma_cpe, beta_cpe,\
                                                                                   gamma1, beta1, eps, X_out, H,   \
                                                                                   nullptr, nullptr)
  if (v4 && C == 64) SFX_CPE4(16, 1);
  else if (v4 && C == 96) SFX_CPE4(8, 3);
  else if (v4 && C == 128) SFX_CPE4(32, 1);
  else if (v4 && C == 256) SFX_CPE4(64, 1);
  else if (v4 && C == 512) SFX_CPE4(64, 2);
  else cpe_residual_ln_kernel<<<sfx::ceil_div(M, 4), 256, 0, st>>>(M, C, T, X, gamma_cpe, beta_cpe, gamma1, beta1, eps,
                                                                   X_out, H);
#undef SFX_CPE4
  return sfx::check_launch("sfx_cpe_residual_ln");
}

// sfx_cpe_residual_ln with T = the centre output of sfx_subm_conv_partials and the pair partials summed per row
// in ascending offset order (pair_pos: sfx_subm_pair_pos; partials: [num_pairs][C], contiguous).  (ABI v15) ldt: T's
// row stride -- C for a per-row centre output, 0 for the conv bias alone when the pair lists carry the centre
// offset (sfx_subm_pairs with_centre: its products are partial rows like every other offset's, summed at k = 13).
int sfx_cpe_residual_ln_pairs(int M, int C, const float* T, long long ldt, const float* partials, const int* pair_pos,
                              long long num_pairs, const float* X, const float* gamma_cpe, const float* beta_cpe,
                              const float* gamma1, const float* beta1, float eps, float* X_out, float* H,
                              void* stream) {
  SFX_REQUIRE(ldt == 0 || ldt == C, "sfx_cpe_residual_ln_pairs: ldt must be C or 0");
  SFX_REQUIRE(M >= 0 && num_pairs >= 0, "sfx_cpe_residual_ln_pairs: bad sizes");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(T && X && gamma_cpe && beta_cpe && gamma1 && beta1 && X_out && H && pair_pos &&
                  (num_pairs == 0 || partials),
              "sfx_cpe_residual_ln_pairs: null buffer");
  SFX_REQUIRE(num_pairs * C * 4 + 64 < 0x7ffffff0ll, "sfx_cpe_residual_ln_pairs: partials exceed 2 GiB");
  const bool v4 = al16(T) && al16(X) && al16(X_out) && al16(H) && al16(gamma_cpe) && al16(beta_cpe) && al16(gamma1) &&
                  al16(beta1) && (!partials || al16(partials));
  SFX_REQUIRE(v4 && (C == 64 || C == 96 || C == 128 || C == 256 || C == 512),
              "sfx_cpe_residual_ln_pairs: needs 16-byte aligned rows and C in {64, 96, 128, 256, 512}");
  hipStream_t st = sfx::as_stream(stream);
#define SFX_CPE4P(G, NV)                                                                                        \
  cpe_residual_ln4_kernel<G, NV, 1><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, T, ldt, X, gamma_cpe, beta_cpe,\
                                                                                  gamma1, beta1, eps, X_out, H,   \
                                                                                  partials, pair_pos)
  if (C == 64) SFX_CPE4P(16, 1);
  else if (C == 96) SFX_CPE4P(8, 3);
  else if (C == 128) SFX_CPE4P(32, 1);
  else if (C == 256) SFX_CPE4P(64, 1);
  else SFX_CPE4P(64, 2);
#undef SFX_CPE4P
  return sfx::check_launch("sfx_cpe_residual_ln_pairs");
}

// (ABI v16) sfx_cpe_residual_ln_pairs with the compacted positions of sfx_subm_pair_lists (pair_cpos [M][32]):
// bit-identical results, fewer position and row loads
int sfx_cpe_residual_ln_cpairs(int M, int C, const float* T, long long ldt, const float* partials,
                               const int* pair_cpos, long long num_pairs, const float* X, const float* gamma_cpe,
                               const float* beta_cpe, const float* gamma1, const float* beta1, float eps, float* X_out,
                               float* H, void* stream) {
  SFX_REQUIRE(ldt == 0 || ldt == C, "sfx_cpe_residual_ln_cpairs: ldt must be C or 0");
  SFX_REQUIRE(M >= 0 && num_pairs >= 0, "sfx_cpe_residual_ln_cpairs: bad sizes");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(T && X && gamma_cpe && beta_cpe && gamma1 && beta1 && X_out && H && pair_cpos &&
                  (num_pairs == 0 || partials),
              "sfx_cpe_residual_ln_cpairs: null buffer");
  SFX_REQUIRE(num_pairs * C * 4 + 64 < 0x7ffffff0ll, "sfx_cpe_residual_ln_cpairs: partials exceed 2 GiB");
  const bool v4 = al16(T) && al16(X) && al16(X_out) && al16(H) && al16(gamma_cpe) && al16(beta_cpe) && al16(gamma1) &&
                  al16(beta1) && (!partials || al16(partials)) && al16(pair_cpos);
  SFX_REQUIRE(v4 && (C == 64 || C == 96 || C == 128 || C == 256 || C == 512),
              "sfx_cpe_residual_ln_cpairs: needs 16-byte aligned rows and C in {64, 96, 128, 256, 512}");
  hipStream_t st = sfx::as_stream(stream);
#define SFX_CPE4C(G, NV)                                                                                        \
  cpe_residual_ln4_kernel<G, NV, 2><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, T, ldt, X, gamma_cpe, beta_cpe,   \
                                                                               gamma1, beta1, eps, X_out, H,      \
                                                                               partials, pair_cpos)
  if (C == 64) SFX_CPE4C(16, 1);
  else if (C == 96) SFX_CPE4C(8, 3);
  else if (C == 128) SFX_CPE4C(32, 1);
  else if (C == 256) SFX_CPE4C(64, 1);
  else SFX_CPE4C(64, 2);
#undef SFX_CPE4C
  return sfx::check_launch("sfx_cpe_residual_ln_cpairs");
}

// (ABI v15) sfx_cpe_residual_ln_pairs + the qkv projection in one launch (eval, C in {64, 96, 128}): X_out = X +
// LN_cpe(T + pair partials), h = LN1(X_out) kept on chip, qkv [M][3C] = h W^T + b with W = sfx_weight_split of the
// qkv weight [3C][C] (w_split, w_inv); max |qkv| published into amax_slot (tag) for sfx_window_attention.
int sfx_cpe_ln_qkv_pairs(int M, int C, const float* T, long long ldt, const float* partials, const int* pair_pos,
                         long long num_pairs, const float* X, const float* gamma_cpe, const float* beta_cpe,
                         const float* gamma1, const float* beta1, float eps, float* X_out, const float* w_split,
                         const float* w_inv, const float* bias, float* qkv, unsigned long long* amax_slot,
                         unsigned tag, void* stream) {
  SFX_REQUIRE(M >= 0 && num_pairs >= 0 && (ldt == 0 || ldt == C), "sfx_cpe_ln_qkv_pairs: bad sizes");
  SFX_REQUIRE(C == 64 || C == 96 || C == 128, "sfx_cpe_ln_qkv_pairs: C must be 64, 96 or 128 (got %d)", C);
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(T && X && gamma_cpe && beta_cpe && gamma1 && beta1 && X_out && pair_pos && w_split && w_inv && bias &&
                  qkv && (num_pairs == 0 || partials) && (!amax_slot || tag != 0),
              "sfx_cpe_ln_qkv_pairs: null buffer");
  SFX_REQUIRE(num_pairs * C * 4 + 64 < 0x7ffffff0ll, "sfx_cpe_ln_qkv_pairs: partials exceed 2 GiB");
  SFX_REQUIRE(al16(T) && al16(X) && al16(X_out) && al16(gamma_cpe) && al16(beta_cpe) && al16(gamma1) &&
                  al16(beta1) && al16(w_split) && al16(w_inv) && al16(bias) && al16(qkv) && (!partials || al16(partials)),
              "sfx_cpe_ln_qkv_pairs: buffers must be 16-byte aligned");
  SFX_REQUIRE(X_out != X, "sfx_cpe_ln_qkv_pairs: in-place output is not supported");
  hipStream_t st = sfx::as_stream(stream);
  const unsigned grid = (unsigned)((M + 127) / 128);
  const uint4* w = reinterpret_cast<const uint4*>(w_split);
#define SFX_LNQKV(G, NV)                                                                                            \
  cpe_ln_qkv_kernel<G, NV><<<grid, 256, 0, st>>>(M, T, ldt, partials, pair_pos, X, gamma_cpe, beta_cpe, gamma1, beta1, \
                                                 eps, X_out, w, w_inv, bias, qkv, amax_slot, tag)
  if (C == 64) SFX_LNQKV(16, 1);
  else if (C == 96) SFX_LNQKV(8, 3);
  else SFX_LNQKV(32, 1);
#undef SFX_LNQKV
  return sfx::check_launch("sfx_cpe_ln_qkv_pairs");
}

}  // extern "C"
