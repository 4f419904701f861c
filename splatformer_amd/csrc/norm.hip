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

}  // namespace

extern "C" {

int sfx_layernorm(int M, int C, const float* X, long long ldx, const float* gamma, const float* beta, float eps,
                  float* Y, long long ldy, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_layernorm: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(X && gamma && beta && Y, "sfx_layernorm: null buffer");
  layernorm_kernel<<<sfx::ceil_div(M, 4), 256, 0, sfx::as_stream(stream)>>>(M, C, X, ldx, gamma, beta, eps, Y, ldy);
  return sfx::check_launch("sfx_layernorm");
}

int sfx_cpe_residual_ln(int M, int C, const float* T, const float* X, const float* gamma_cpe, const float* beta_cpe,
                        const float* gamma1, const float* beta1, float eps, float* X_out, float* H, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_cpe_residual_ln: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(T && X && gamma_cpe && beta_cpe && gamma1 && beta1 && X_out && H, "sfx_cpe_residual_ln: null buffer");
  cpe_residual_ln_kernel<<<sfx::ceil_div(M, 4), 256, 0, sfx::as_stream(stream)>>>(M, C, T, X, gamma_cpe, beta_cpe,
                                                                                   gamma1, beta1, eps, X_out, H);
  return sfx::check_launch("sfx_cpe_residual_ln");
}

}  // extern "C"
