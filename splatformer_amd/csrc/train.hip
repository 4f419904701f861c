// Training-mode kernels of the refiner (configs C/D): the backward of the row/column normalisations,
// the pooling reductions and the drop-path / activation terms, train-mode BatchNorm, and the optimiser.
//
// Reference semantics (autograd of the modules the reference trains, train.py:240-303):
// - nn.LayerNorm backward (Block.norm1/norm2, cpe.2), biased variance, eps 1e-5;
// - nn.BatchNorm1d(eps=1e-3, momentum=0.01) in train mode (batch statistics, running-stat update with the
//   unbiased variance) -- SyncBatchNorm under DDP (train.py:404): the per-column sums are produced here
//   and all-reduced by the caller between the reduce and the finalize/apply kernels;
// - torch_scatter segment_csr(max) backward (SerializedPooling): the gradient goes to the arg-max row;
// - torch.optim.Adam (train.py:301, utils/optimizers.py, eps 1e-15) after clip_grad_norm_(2.0).
// All column reductions are two-level and deterministic (fp64 partials, fixed order).
#include "common.h"

namespace {

constexpr int MAXV = 8;  // LayerNorm rows: C <= 512

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_g(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * expf(-0.5f * x * x);
}

// ---- LayerNorm backward -------------------------------------------------------------------------------
// dX = rstd * (gy - mean(gy) - xhat * mean(gy * xhat)),  gy = dY * gamma
__device__ __forceinline__ void ln_bwd_row(const float* x, const float* dy, int C, int lane,
                                           const float* __restrict__ g, float eps, float* dx) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (lane + 64 * i < C) s += x[i];
  const float mean = sfx::wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (lane + 64 * i < C) {
      const float d = x[i] - mean;
      q += d * d;
    }
  const float rstd = 1.f / sqrtf(sfx::wave_sum(q) / (float)C + eps);
  float a = 0.f, b = 0.f;
  float xh[MAXV], gy[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    xh[i] = (x[i] - mean) * rstd;
    gy[i] = c < C ? dy[i] * g[c] : 0.f;
    if (c < C) {
      a += gy[i];
      b += gy[i] * xh[i];
    }
  }
  a = sfx::wave_sum(a) / (float)C;
  b = sfx::wave_sum(b) / (float)C;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) dx[i] = rstd * (gy[i] - a - xh[i] * b);
}

__global__ void __launch_bounds__(256) layernorm_bwd_kernel(int M, int C, const float* __restrict__ X, long long ldx,
                                                            const float* __restrict__ g, const float* __restrict__ dY,
                                                            long long ldgy, const float* __restrict__ dR,
                                                            long long ldr, float eps, float* __restrict__ dX,
                                                            long long lddx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  float x[MAXV], dy[MAXV], dx[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    x[i] = c < C ? X[(long long)row * ldx + c] : 0.f;
    dy[i] = c < C ? dY[(long long)row * ldgy + c] : 0.f;
  }
  ln_bwd_row(x, dy, C, lane, g, eps, dx);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) dX[(long long)row * lddx + c] = dx[i] + (dR ? dR[(long long)row * ldr + c] : 0.f);
  }
}

// Block tail backward: dX1 = dX2 + LN1'(X1, dH);  dU = LN_cpe'(U, dX1)
__global__ void __launch_bounds__(256) cpe_ln_bwd_kernel(int M, int C, const float* __restrict__ U,
                                                         const float* __restrict__ X1, const float* __restrict__ g_cpe,
                                                         const float* __restrict__ g1, const float* __restrict__ dX2,
                                                         const float* __restrict__ dH, float eps,
                                                         float* __restrict__ dX1, float* __restrict__ dU) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const long long o = (long long)row * C;
  float x[MAXV], dy[MAXV], d1[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    x[i] = c < C ? X1[o + c] : 0.f;
    dy[i] = c < C ? dH[o + c] : 0.f;
  }
  ln_bwd_row(x, dy, C, lane, g1, eps, d1);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    d1[i] += c < C ? dX2[o + c] : 0.f;
    x[i] = c < C ? U[o + c] : 0.f;
  }
  float du[MAXV];
  ln_bwd_row(x, d1, C, lane, g_cpe, eps, du);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      dX1[o + c] = d1[i];
      dU[o + c] = du[i];
    }
  }
}

// Vectorised forms for C in {64, 96, 128, 256, 512} (norm.hip's layout): a row is held by G lanes, NV float4 per
// lane, 64/G rows per wave -- 16-byte loads and log2(G)-step group reductions instead of one wave per row with
// 4-byte loads and full-wave reductions (C = 64: 4x fewer reduction steps per row, no idle lanes).
template <int G>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int G, int NV>
__device__ __forceinline__ void ln_bwd_row4(const float4 (&x)[NV], const float4 (&dy)[NV], const float* __restrict__ g,
                                            float eps, int sub, float4 (&dx)[NV]) {
  constexpr float inv_c = 1.f / (float)(4 * G * NV);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (x[i].x + x[i].y) + (x[i].z + x[i].w);
  const float mean = gsum<G>(s) * inv_c;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a = x[i].x - mean, b = x[i].y - mean, c = x[i].z - mean, d = x[i].w - mean;
    q += (a * a + b * b) + (c * c + d * d);
  }
  const float rstd = 1.f / sqrtf(gsum<G>(q) * inv_c + eps);
  float4 xh[NV], gy[NV];
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 gg = *reinterpret_cast<const float4*>(g + 4 * (sub + G * i));
    xh[i] = make_float4((x[i].x - mean) * rstd, (x[i].y - mean) * rstd, (x[i].z - mean) * rstd,
                        (x[i].w - mean) * rstd);
    gy[i] = make_float4(dy[i].x * gg.x, dy[i].y * gg.y, dy[i].z * gg.z, dy[i].w * gg.w);
    a += (gy[i].x + gy[i].y) + (gy[i].z + gy[i].w);
    b += (gy[i].x * xh[i].x + gy[i].y * xh[i].y) + (gy[i].z * xh[i].z + gy[i].w * xh[i].w);
  }
  a = gsum<G>(a) * inv_c;
  b = gsum<G>(b) * inv_c;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    dx[i] = make_float4(rstd * (gy[i].x - a - xh[i].x * b), rstd * (gy[i].y - a - xh[i].y * b),
                        rstd * (gy[i].z - a - xh[i].z * b), rstd * (gy[i].w - a - xh[i].w * b));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int G, int NV>
__global__ void __launch_bounds__(256) layernorm_bwd4_kernel(int M, const float* __restrict__ X, long long ldx,
                                                             const float* __restrict__ g, const float* __restrict__ dY,
                                                             long long ldgy, const float* __restrict__ dR,
                                                             long long ldr, float eps, float* __restrict__ dX,
                                                             long long lddx) {
  const int row = blockIdx.x * (256 / G) + threadIdx.x / G;
  const int sub = threadIdx.x % G;
  if (row >= M) return;
  float4 x[NV], dy[NV], dx[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    x[i] = *reinterpret_cast<const float4*>(X + (long long)row * ldx + 4 * (sub + G * i));
    dy[i] = *reinterpret_cast<const float4*>(dY + (long long)row * ldgy + 4 * (sub + G * i));
  }
  ln_bwd_row4<G, NV>(x, dy, g, eps, sub, dx);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float4 o = dx[i];
    if (dR) o = add4(o, *reinterpret_cast<const float4*>(dR + (long long)row * ldr + 4 * (sub + G * i)));
    *reinterpret_cast<float4*>(dX + (long long)row * lddx + 4 * (sub + G * i)) = o;
  }
}

template <int G, int NV>
__global__ void __launch_bounds__(256) cpe_ln_bwd4_kernel(int M, const float* __restrict__ U,
                                                          const float* __restrict__ X1, const float* __restrict__ g_cpe,
                                                          const float* __restrict__ g1, const float* __restrict__ dX2,
                                                          const float* __restrict__ dH, float eps,
                                                          float* __restrict__ dX1, float* __restrict__ dU) {
  constexpr int C = 4 * G * NV;
  const int row = blockIdx.x * (256 / G) + threadIdx.x / G;
  const int sub = threadIdx.x % G;
  if (row >= M) return;
  const long long o = (long long)row * C;
  float4 x[NV], dy[NV], d1[NV], du[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    x[i] = *reinterpret_cast<const float4*>(X1 + o + 4 * (sub + G * i));
    dy[i] = *reinterpret_cast<const float4*>(dH + o + 4 * (sub + G * i));
  }
  ln_bwd_row4<G, NV>(x, dy, g1, eps, sub, d1);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    d1[i] = add4(d1[i], *reinterpret_cast<const float4*>(dX2 + o + 4 * (sub + G * i)));
    x[i] = *reinterpret_cast<const float4*>(U + o + 4 * (sub + G * i));
  }
  ln_bwd_row4<G, NV>(x, d1, g_cpe, eps, sub, du);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    *reinterpret_cast<float4*>(dX1 + o + 4 * (sub + G * i)) = d1[i];
    *reinterpret_cast<float4*>(dU + o + 4 * (sub + G * i)) = du[i];
  }
}

__host__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ---- column reductions (BatchNorm statistics and its backward sums) ------------------------------------
// 128 rows per workgroup: M / 128 workgroups (782 at 100k rows, > 3 per CU) with 8 independent loads in flight per
// thread -- at 512 rows (196 workgroups for 100k rows, each thread a chain of 128 dependent-latency loads) the
// reductions ran at ~0.3 of HBM bandwidth (12.6 ms per config-C step, profiles/r05_configC_kernel_top.txt)
constexpr int COL_BLOCK_ROWS = 128;

// mode 0: (sum x, sum x^2);  mode 1: (sum g, sum g*xhat) with g = dY * act'(BN(x)), xhat = (x-mean)*rstd
__global__ void __launch_bounds__(256) colsum2_kernel(int mode, int M, int C, const float* __restrict__ X,
                                                      long long ldx, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int act,
                                                      const float* __restrict__ dY, long long ldgy,
                                                      double* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  const int m0 = blockIdx.y * COL_BLOCK_ROWS, m1 = min(M, m0 + COL_BLOCK_ROWS);
  double s0 = 0.0, s1 = 0.0;
  if (c < C) {
    if (mode == 0) {
#pragma unroll 8
      for (int m = m0 + sub; m < m1; m += 4) {
        const double v = X[(long long)m * ldx + c];
        s0 += v;
        s1 += v * v;
      }
    } else {
      const float mu = mean[c], rs = rstd[c], ga = gamma[c], be = beta[c];
#pragma unroll 8
      for (int m = m0 + sub; m < m1; m += 4) {
        const float xh = (X[(long long)m * ldx + c] - mu) * rs;
        float g = dY[(long long)m * ldgy + c];
        if (act == 1) g *= gelu_g(xh * ga + be);
        s0 += g;
        s1 += (double)g * xh;
      }
    }
  }
  __shared__ double red[2][4][64];
  red[0][sub][threadIdx.x & 63] = s0;
  red[1][sub][threadIdx.x & 63] = s1;
  __syncthreads();
  if (sub == 0 && c < C) {
    const int l = threadIdx.x;
    part[(long long)blockIdx.y * 2 * C + c] = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
    part[(long long)blockIdx.y * 2 * C + C + c] = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
  }
}

// one wave per output column: lanes take the partial rows lane, lane+64, ... (fixed order), then a fixed
// butterfly -- deterministic, and 2C waves of parallelism instead of 2C threads
__global__ void __launch_bounds__(256) colsum2_final_kernel(int C, int blocks, const double* __restrict__ part,
                                                            double* __restrict__ out) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= 2 * C) return;
  double s = 0.0;
  for (int b = lane; b < blocks; b += 64) s += part[(long long)b * 2 * C + j];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[j] = s;
}

// mean, biased var -> rstd; scale = gamma*rstd, shift = beta - mean*scale; running stats (unbiased var)
__global__ void bn_finalize_kernel(int C, double count, const double* __restrict__ sums, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum,
                                   float* __restrict__ running_mean, float* __restrict__ running_var,
                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                   float* __restrict__ scale_out, float* __restrict__ shift_out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float mf = (float)mean;
  mean_out[c] = mf;
  rstd_out[c] = rstd;
  const float sc = gamma[c] * rstd;
  scale_out[c] = sc;
  shift_out[c] = beta[c] - mf * sc;
  if (running_mean) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mf;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

// Y = act(X*scale + shift) (+ R[ridx[m]])   (train-mode BN apply; unpooling residual)
__global__ void __launch_bounds__(256) affine_act_kernel(int M, int C, const float* __restrict__ X, long long ldx,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int act,
                                                         const float* __restrict__ R, long long ldr,
                                                         const int* __restrict__ ridx, float* __restrict__ Y,
                                                         long long ldy) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)M * C) return;
  const int m = (int)(e / C), c = (int)(e - (long long)m * C);
  float v = X[(long long)m * ldx + c] * scale[c] + shift[c];
  if (act == 1) v = gelu_f(v);
  if (R) v += R[(long long)(ridx ? ridx[m] : m) * ldr + c];
  Y[(long long)m * ldy + c] = v;
}

// dX (=|+=) gamma*rstd*(g - S0/count - xhat*S1/count)
__global__ void __launch_bounds__(256) bn_act_bwd_apply_kernel(int M, int C, const float* __restrict__ X, long long ldx,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, int act,
                                                               const float* __restrict__ dY, long long ldgy,
                                                               const double* __restrict__ sums, double count,
                                                               float* __restrict__ dX, long long lddx, int accumulate) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)M * C) return;
  const int m = (int)(e / C), c = (int)(e - (long long)m * C);
  const float xh = (X[(long long)m * ldx + c] - mean[c]) * rstd[c];
  float g = dY[(long long)m * ldgy + c];
  if (act == 1) g *= gelu_g(xh * gamma[c] + beta[c]);
  const float a = (float)(sums[c] / count), b = (float)(sums[C + c] / count);
  const float v = gamma[c] * rstd[c] * (g - a - xh * b);
  float* d = dX + (long long)m * lddx + c;
  *d = accumulate ? *d + v : v;
}

// ---- pooling reductions --------------------------------------------------------------------------------
// segment max over sorted runs with the arg-max row (first maximum in run order: torch_scatter segment_csr)
__global__ void segment_max_arg_kernel(int m, int C, const int* __restrict__ idx_ptr, const int* __restrict__ sidx,
                                       const float* __restrict__ X, float* __restrict__ Y, int* __restrict__ arg) {
  const int s = blockIdx.x;
  const int beg = idx_ptr[s], end = idx_ptr[s + 1];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v = -INFINITY;
    int a = -1;
    for (int p = beg; p < end; ++p) {
      const int r = sidx[p];
      const float x = X[(long long)r * C + c];
      if (x > v || a < 0) {
        v = x;
        a = r;
      }
    }
    Y[(long long)s * C + c] = v;
    arg[(long long)s * C + c] = a;
  }
}

__global__ void __launch_bounds__(256) segment_max_bwd_kernel(int m, int C, const float* __restrict__ dY,
                                                              const int* __restrict__ arg, float* __restrict__ dX) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)m * C) return;
  const int c = (int)(e % C);
  const int r = arg[e];
  if (r >= 0) dX[(long long)r * C + c] = dY[e];
}

// Y[s] = sum of X rows of run s (backward of the unpooling gather feat[inverse])
__global__ void segment_sum_kernel(int m, int C, const int* __restrict__ idx_ptr, const int* __restrict__ sidx,
                                   const float* __restrict__ X, long long ldx, float* __restrict__ Y) {
  const int s = blockIdx.x;
  const int beg = idx_ptr[s], end = idx_ptr[s + 1];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v = 0.f;
    for (int p = beg; p < end; ++p) v += X[(long long)sidx[p] * ldx + c];
    Y[(long long)s * C + c] = v;
  }
}

// dX = dY * act'(pre) for cols < ncols (1 GELU on pre-act, 2 ReLU, 3 tanh given its output), dY elsewhere
__global__ void __launch_bounds__(256) act_bwd_kernel(int M, int N, const float* __restrict__ dY, long long ldgy,
                                                      const float* __restrict__ pre, long long ldp, int act, int ncols,
                                                      float* __restrict__ dX, long long lddx) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)M * N) return;
  const int m = (int)(e / N), c = (int)(e - (long long)m * N);
  float g = dY[(long long)m * ldgy + c];
  if (c < ncols) {
    const float p = pre[(long long)m * ldp + c];
    g *= act == 1 ? gelu_g(p) : act == 2 ? (p > 0.f ? 1.f : 0.f) : 1.f - p * p;
  }
  dX[(long long)m * lddx + c] = g;
}

// ---- DropPath keep masks ------------------------------------------------------------------------------
// timm DropPath per point (reference pointtransformer_v3.py:145, drop_path=0.3 schedule): out[i] = 1/keep when
// u_i < keep, else 0, with u_i uniform on [0, 1) in 2^-24 steps from a counter-based hash of (seed, i) (splitmix64
// finaliser) -- one launch per mask instead of torch's rand + compare + cast + scale.
__global__ void __launch_bounds__(256) drop_mask_kernel(long long n, float keep, unsigned long long seed,
                                                        float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  unsigned long long z = seed + (unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.f / 16777216.f);
  out[i] = u < keep ? 1.f / keep : 0.f;
}

// ---- optimiser -----------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sumsq_kernel(long long n, const float* __restrict__ x, double* __restrict__ out) {
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = x[i];
    s += v * v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

// clip_grad_norm_: coef = min(1, max_norm / (||g|| + 1e-6))
__global__ void clip_coef_kernel(const double* __restrict__ sumsq, float max_norm, float* __restrict__ coef,
                                 float* __restrict__ norm_out) {
  const float norm = (float)sqrt(*sumsq);
  if (norm_out) *norm_out = norm;
  const float c = max_norm / (norm + 1e-6f);
  *coef = c < 1.f ? c : 1.f;
}

// torch.optim.Adam (single tensor math; weight_decay folded into the gradient)
__global__ void __launch_bounds__(256) adam_kernel(long long n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m1, float* __restrict__ m2,
                                                   const float* __restrict__ gscale, float lr, float beta1,
                                                   float beta2, float eps, float weight_decay, float bc1,
                                                   float bc2_sqrt) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float gr = g[i] * (gscale ? *gscale : 1.f);
  if (weight_decay != 0.f) gr += weight_decay * p[i];
  const float a = m1[i] + (1.f - beta1) * (gr - m1[i]);
  const float b = beta2 * m2[i] + (1.f - beta2) * gr * gr;
  m1[i] = a;
  m2[i] = b;
  const float denom = sqrtf(b) / bc2_sqrt + eps;
  p[i] -= (lr / bc1) * a / denom;
}

}  // namespace

extern "C" {

int sfx_layernorm_bwd(int M, int C, const float* X, long long ldx, const float* gamma, const float* dY,
                      long long ldgy, const float* dR, long long ldr, float eps, float* dX, long long lddx,
                      void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_layernorm_bwd: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(X && gamma && dY && dX, "sfx_layernorm_bwd: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const bool v4 = al16(X) && al16(gamma) && al16(dY) && al16(dX) && (!dR || al16(dR)) && ldx % 4 == 0 &&
                  ldgy % 4 == 0 && lddx % 4 == 0 && (!dR || ldr % 4 == 0);
#define SFX_LNB4(G, NV)                                                                                      \
  layernorm_bwd4_kernel<G, NV><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, X, ldx, gamma, dY, ldgy, dR, ldr, \
                                                                          eps, dX, lddx)
  if (v4 && C == 64) SFX_LNB4(16, 1);
  else if (v4 && C == 96) SFX_LNB4(8, 3);
  else if (v4 && C == 128) SFX_LNB4(32, 1);
  else if (v4 && C == 256) SFX_LNB4(64, 1);
  else if (v4 && C == 512) SFX_LNB4(64, 2);
  else
    layernorm_bwd_kernel<<<sfx::ceil_div(M, 4), 256, 0, st>>>(M, C, X, ldx, gamma, dY, ldgy, dR, ldr, eps, dX, lddx);
#undef SFX_LNB4
  return sfx::check_launch("sfx_layernorm_bwd");
}

int sfx_cpe_ln_bwd(int M, int C, const float* U, const float* X1, const float* gamma_cpe, const float* gamma1,
                   const float* dX2, const float* dH, float eps, float* dX1, float* dU, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && C <= 64 * MAXV, "sfx_cpe_ln_bwd: C must be in [1, 512]");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(U && X1 && gamma_cpe && gamma1 && dX2 && dH && dX1 && dU, "sfx_cpe_ln_bwd: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const bool v4 = al16(U) && al16(X1) && al16(gamma_cpe) && al16(gamma1) && al16(dX2) && al16(dH) && al16(dX1) &&
                  al16(dU);
#define SFX_CPEB4(G, NV)                                                                                       \
  cpe_ln_bwd4_kernel<G, NV><<<sfx::ceil_div(M, 256 / G), 256, 0, st>>>(M, U, X1, gamma_cpe, gamma1, dX2, dH, eps, \
                                                                       dX1, dU)
  if (v4 && C == 64) SFX_CPEB4(16, 1);
  else if (v4 && C == 96) SFX_CPEB4(8, 3);
  else if (v4 && C == 128) SFX_CPEB4(32, 1);
  else if (v4 && C == 256) SFX_CPEB4(64, 1);
  else if (v4 && C == 512) SFX_CPEB4(64, 2);
  else
    cpe_ln_bwd_kernel<<<sfx::ceil_div(M, 4), 256, 0, st>>>(M, C, U, X1, gamma_cpe, gamma1, dX2, dH, eps, dX1, dU);
#undef SFX_CPEB4
  return sfx::check_launch("sfx_cpe_ln_bwd");
}

size_t sfx_colsum2_workspace_bytes(int M, int C) {
  return (size_t)sfx::ceil_div(M > 0 ? M : 1, COL_BLOCK_ROWS) * 2 * (size_t)C * sizeof(double);
}

static int colsum2(int mode, int M, int C, const float* X, long long ldx, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, int act, const float* dY, long long ldgy, void* ws,
                   size_t ws_bytes, double* sums, hipStream_t st, const char* what) {
  SFX_REQUIRE(M >= 1 && C > 0, "%s: bad sizes", what);
  SFX_REQUIRE(ws && ws_bytes >= sfx_colsum2_workspace_bytes(M, C), "%s: workspace too small", what);
  const int blocks = (int)sfx::ceil_div(M, COL_BLOCK_ROWS);
  colsum2_kernel<<<dim3(sfx::ceil_div(C, 64), blocks), 256, 0, st>>>(mode, M, C, X, ldx, mean, rstd, gamma, beta, act,
                                                                      dY, ldgy, static_cast<double*>(ws));
  colsum2_final_kernel<<<sfx::ceil_div(2 * C, 4), 256, 0, st>>>(C, blocks, static_cast<double*>(ws), sums);
  return sfx::check_launch(what);
}

int sfx_bn_stats(int M, int C, const float* X, long long ldx, void* ws, size_t ws_bytes, double* sums,
                 void* stream) {
  SFX_REQUIRE(X && sums, "sfx_bn_stats: null buffer");
  return colsum2(0, M, C, X, ldx, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, ws, ws_bytes, sums,
                 sfx::as_stream(stream), "sfx_bn_stats");
}

int sfx_bn_finalize(int C, double count, const double* sums, const float* gamma, const float* beta, float eps,
                    float momentum, float* running_mean, float* running_var, float* mean_out, float* rstd_out,
                    float* scale_out, float* shift_out, void* stream) {
  SFX_REQUIRE(C > 0 && count >= 1.0, "sfx_bn_finalize: bad sizes");
  SFX_REQUIRE(sums && gamma && beta && mean_out && rstd_out && scale_out && shift_out &&
                  (!running_mean == !running_var),
              "sfx_bn_finalize: null buffer");
  bn_finalize_kernel<<<sfx::ceil_div(C, 256), 256, 0, sfx::as_stream(stream)>>>(
      C, count, sums, gamma, beta, eps, momentum, running_mean, running_var, mean_out, rstd_out, scale_out, shift_out);
  return sfx::check_launch("sfx_bn_finalize");
}

int sfx_affine_act(int M, int C, const float* X, long long ldx, const float* scale, const float* shift, int act,
                   const float* R, long long ldr, const int* ridx, float* Y, long long ldy, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && (act == 0 || act == 1), "sfx_affine_act: bad args");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(X && scale && shift && Y, "sfx_affine_act: null buffer");
  affine_act_kernel<<<sfx::ceil_div((long long)M * C, 256), 256, 0, sfx::as_stream(stream)>>>(
      M, C, X, ldx, scale, shift, act, R, ldr, ridx, Y, ldy);
  return sfx::check_launch("sfx_affine_act");
}

int sfx_bn_act_bwd_reduce(int M, int C, const float* X, long long ldx, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, const float* dY, long long ldgy, void* ws,
                          size_t ws_bytes, double* sums, void* stream) {
  SFX_REQUIRE(X && mean && rstd && gamma && beta && dY && sums, "sfx_bn_act_bwd_reduce: null buffer");
  SFX_REQUIRE(act == 0 || act == 1, "sfx_bn_act_bwd_reduce: bad act");
  return colsum2(1, M, C, X, ldx, mean, rstd, gamma, beta, act, dY, ldgy, ws, ws_bytes, sums, sfx::as_stream(stream),
                 "sfx_bn_act_bwd_reduce");
}

int sfx_bn_act_bwd_apply(int M, int C, const float* X, long long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, int act, const float* dY, long long ldgy,
                         const double* sums, double count, float* dX, long long lddx, int accumulate, void* stream) {
  SFX_REQUIRE(M >= 0 && C > 0 && count >= 1.0 && (act == 0 || act == 1), "sfx_bn_act_bwd_apply: bad args");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(X && mean && rstd && gamma && beta && dY && sums && dX, "sfx_bn_act_bwd_apply: null buffer");
  bn_act_bwd_apply_kernel<<<sfx::ceil_div((long long)M * C, 256), 256, 0, sfx::as_stream(stream)>>>(
      M, C, X, ldx, mean, rstd, gamma, beta, act, dY, ldgy, sums, count, dX, lddx, accumulate);
  return sfx::check_launch("sfx_bn_act_bwd_apply");
}

int sfx_segment_max_arg(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X, float* Y, int* arg,
                        void* stream) {
  SFX_REQUIRE(m >= 0 && C > 0, "sfx_segment_max_arg: bad args");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(idx_ptr && sorted_idx && X && Y && arg, "sfx_segment_max_arg: null buffer");
  const int threads = C >= 256 ? 256 : (C >= 128 ? 128 : 64);
  segment_max_arg_kernel<<<m, threads, 0, sfx::as_stream(stream)>>>(m, C, idx_ptr, sorted_idx, X, Y, arg);
  return sfx::check_launch("sfx_segment_max_arg");
}

int sfx_segment_max_bwd(int m, int C, const float* dY, const int* arg, float* dX, void* stream) {
  SFX_REQUIRE(m >= 0 && C > 0, "sfx_segment_max_bwd: bad args");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(dY && arg && dX, "sfx_segment_max_bwd: null buffer");
  segment_max_bwd_kernel<<<sfx::ceil_div((long long)m * C, 256), 256, 0, sfx::as_stream(stream)>>>(m, C, dY, arg, dX);
  return sfx::check_launch("sfx_segment_max_bwd");
}

int sfx_segment_sum(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X, long long ldx, float* Y,
                    void* stream) {
  SFX_REQUIRE(m >= 0 && C > 0, "sfx_segment_sum: bad args");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(idx_ptr && sorted_idx && X && Y, "sfx_segment_sum: null buffer");
  const int threads = C >= 256 ? 256 : (C >= 128 ? 128 : 64);
  segment_sum_kernel<<<m, threads, 0, sfx::as_stream(stream)>>>(m, C, idx_ptr, sorted_idx, X, ldx, Y);
  return sfx::check_launch("sfx_segment_sum");
}

int sfx_act_bwd(int M, int N, const float* dY, long long ldgy, const float* pre, long long ldp, int act, int ncols,
                float* dX, long long lddx, void* stream) {
  SFX_REQUIRE(M >= 0 && N > 0 && act >= 1 && act <= 3, "sfx_act_bwd: bad args");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(dY && pre && dX, "sfx_act_bwd: null buffer");
  act_bwd_kernel<<<sfx::ceil_div((long long)M * N, 256), 256, 0, sfx::as_stream(stream)>>>(M, N, dY, ldgy, pre, ldp,
                                                                                           act, ncols, dX, lddx);
  return sfx::check_launch("sfx_act_bwd");
}

int sfx_sumsq(long long n, const float* x, double* out, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_sumsq: bad size");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(x && out, "sfx_sumsq: null buffer");
  long long blocks = sfx::ceil_div(n, 256 * 8);
  if (blocks > 1024) blocks = 1024;
  sumsq_kernel<<<(unsigned)blocks, 256, 0, sfx::as_stream(stream)>>>(n, x, out);
  return sfx::check_launch("sfx_sumsq");
}

int sfx_clip_coef(const double* sumsq, float max_norm, float* coef, float* norm_out, void* stream) {
  SFX_REQUIRE(sumsq && coef, "sfx_clip_coef: null buffer");
  clip_coef_kernel<<<1, 1, 0, sfx::as_stream(stream)>>>(sumsq, max_norm, coef, norm_out);
  return sfx::check_launch("sfx_clip_coef");
}

int sfx_drop_mask(long long n, float keep, unsigned long long seed, float* out, void* stream) {
  SFX_REQUIRE(n >= 0 && keep > 0.f && keep <= 1.f, "sfx_drop_mask: bad args");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(out, "sfx_drop_mask: null buffer");
  drop_mask_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, keep, seed, out);
  return sfx::check_launch("sfx_drop_mask");
}

int sfx_adam_step(long long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  const float* grad_scale, float lr, float beta1, float beta2, float eps, float weight_decay,
                  int step, void* stream) {
  SFX_REQUIRE(n >= 0 && step >= 1, "sfx_adam_step: bad args");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(param && grad && exp_avg && exp_avg_sq, "sfx_adam_step: null buffer");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  adam_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, param, grad, exp_avg, exp_avg_sq,
                                                                          grad_scale, lr, beta1, beta2, eps,
                                                                          weight_decay, (float)bc1,
                                                                          (float)sqrt(bc2));
  return sfx::check_launch("sfx_adam_step");
}

}  // extern "C"
