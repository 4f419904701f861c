// FeaturePredictor output heads + residual in one launch (reference models/feature_predictor.py:74-94, :201-235):
//   y = cat(backbone [N, 96], feat [N, Cin]);  per feature f: o_f = L4(ReLU(L3(ReLU(L2(ReLU(L1(y)))))))
//   (Linear 119 -> 128 -> 128 -> 128 -> c_f), tanh on the means head, out_f = feat_f + o_f.
//
// The unfused form (one GEMM for the six first layers, two block-diagonal grouped GEMMs, one block-diagonal output
// GEMM) writes and re-reads the [N, 768] hidden activation three times: ~1.5 GB per 100k-point refine.  Here every
// hidden activation stays in registers; HBM traffic is the [N, 120] input read and the [N, Cin] output write.
//
// Arithmetic: fp32-accurate fp16x2 MFMA (gemm.hip's scheme: every operand a power-of-two scaled pair of fp16 terms
// h + l, every 32x32x16 block h*h + h*l + l*h on v_mfma_f32_32x32x16_f16, fp32 accumulation).  Scales: the input
// row and every hidden row (all 128 units of one head, per point) by their exact maxima into [2^14, 2^15); weight
// rows by their own maxima (pre-split once per weight version, sfx_heads_pack).  The last layer (c_f <= 45 outputs)
// runs on the VALU in fp32 from the unrounded ReLU outputs.
//
// Work decomposition (mlp.hip's dataflow): one workgroup = 8 waves x 32 points, points on the lanes.  A layer is
// computed transposed, hid^T[128 units, 32 points] = W . x^T: the weights are the A operand (streamed through an
// LDS ring by LDS-DMA, 16 KB phases = one 32-deep k-chunk for all 4 unit blocks), the activation the B operand in
// registers: the input row's fragments (kept for all heads) for the first layer, the previous layer's accumulator
// registers for the others (a 32x32 accumulator's registers 8s..8s+7 are the k-step-s B fragment with the k order
// permuted, cdna_hip_programming.md §3 -- sfx_heads_pack lays the weights out in that order).
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace {

using namespace sfxg;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int HW = 128;               // head width (feature_predictor.py:74: width 128)
constexpr int MAXH = 6;               // heads
constexpr int SLAB = 8192;            // [2 unit blocks][2 terms][32 rows][32 positions] fp16
constexpr int PHASE = 2 * SLAB;
constexpr int WAVES = 8;
#ifndef SFX_HEADS_RING
#define SFX_HEADS_RING 4
#endif
constexpr int RING = SFX_HEADS_RING;  // LDS ring phases
constexpr int PIECES = PHASE / 1024 / WAVES;  // 1 KB LDS-DMA pieces per wave per phase

struct HeadsArgs {
  int ng;              // heads
  int kin;             // input columns read (backbone width + Cin)
  int out_dim;         // packed output width = sum of head widths
  int res_off;         // column of the residual record in the input row
  int n_tanh;          // leading output columns with tanh (the means head)
  int ocol[MAXH + 1];  // output column of head g (ocol[ng] = out_dim)
};

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
__device__ __forceinline__ int slab_off(int r, int q) {
  return r * 64 + ((((q >> 3) ^ (r >> 2)) & 3) << 4) + ((q & 7) << 1);
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

// params (floats): [(g*3 + L) * 256 + 2 * ((ob * 2 + h) * 16 + i)] = (1/s_u, b_u) of unit u = 32 ob + acc_row(i, h)
// of layer L of head g; then W4 rows (out_dim x 128, natural order) at W4_OFF; then b4 (out_dim) at B4_OFF.
constexpr int W4_OFF = MAXH * 3 * 256;
__host__ __device__ constexpr int b4_off(int out_dim) { return W4_OFF + out_dim * HW; }

template <int KP>
__global__ void __launch_bounds__(WAVES * 64, 1)
heads_kernel(int M, const float* __restrict__ X, long long ldx, const float* __restrict__ stream,
             const float* __restrict__ par, int npar, HeadsArgs a, float* __restrict__ Y, int gper) {
  constexpr int NT = KP / 16;       // 16-deep k-steps of the input
  constexpr int KC0 = KP / 32;      // first-layer k-chunks (phases)
  constexpr int PPH = KC0 + 8;      // phases per head
  // heads [g0, g1) of this workgroup's points (blockIdx.y: head group; disjoint output columns, no combine)
  const int g0 = (int)blockIdx.y * gper, g1 = min(a.ng, g0 + gper);
  __shared__ __attribute__((aligned(16))) char lds[RING * PHASE];
  extern __shared__ float s_par[];  // npar floats (dynamic LDS)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int prow = (int)blockIdx.x * (WAVES * 32) + wid * 32 + r32;
  const bool pok = prow < M;
  const int P0 = g0 * PPH, NP = g1 * PPH;  // this workgroup's phases of the weight stream

  const char* gstream = reinterpret_cast<const char*>(stream);
  auto issue = [&](int q) {
    const char* src = gstream + (size_t)q * PHASE + wid * (PIECES * 1024) + lane * 16;
    char* dst = lds + (q % RING) * PHASE + wid * (PIECES * 1024);
#pragma unroll
    for (int pc = 0; pc < PIECES; ++pc)
      __builtin_amdgcn_global_load_lds(src + pc * 1024, (__attribute__((address_space(3))) void*)(dst + pc * 1024),
                                       16, 0, 0);
  };
#pragma unroll
  for (int q = 0; q < RING - 1; ++q)
    if (P0 + q < NP) issue(P0 + q);

  for (int i = tid; i < npar; i += WAVES * 64) s_par[i] = par[i];

  // ---- the point's input row: channels 16 t + 8 h + 0..7 of k-step t, zero past kin ----
  const __amdgpu_buffer_rsrc_t rX = rsrc_ext(X, (unsigned)M * (unsigned)ldx * 4u);
  const unsigned xr = (unsigned)prow * (unsigned)ldx;
  f16x8 xb[NT][2];
  float in_inv;  // 1 / the input row's scale
  {
    float4 v[2 * NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 16 * t + 8 * h + 4 * u;
        float4 w = bload4(rX, pok && c < a.kin ? (xr + (unsigned)c) * 4u : OOB);
        if (c + 4 > a.kin) {  // (a row's tail past kin: the next row's columns or padding)
          if (c + 0 >= a.kin) w.x = 0.f;
          if (c + 1 >= a.kin) w.y = 0.f;
          if (c + 2 >= a.kin) w.z = 0.f;
          if (c + 3 >= a.kin) w.w = 0.f;
        }
        v[2 * t + u] = w;
      }
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i)
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const int e = (mx > 0.f && mx <= 3.4028235e38f) ? row_exp(mx) + 2 : 0;
    const float sc = ldexpf(1.f, e);
    in_inv = ldexpf(1.f, -e);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      uint2 lo[2], hi[2];
      split2h(v[2 * t], sc, lo);
      split2h(v[2 * t + 1], sc, hi);
      xb[t][0] = __builtin_bit_cast(f16x8, make_uint4(lo[0].x, lo[0].y, hi[0].x, hi[0].y));
      xb[t][1] = __builtin_bit_cast(f16x8, make_uint4(lo[1].x, lo[1].y, hi[1].x, hi[1].y));
    }
  }
  float act_inv = in_inv;  // 1 / scale of the current B operand (the input row, then each hidden row)
  __syncthreads();  // s_par visible (only plain stores and in-flight DMAs precede it; the DMAs are waited below)

  floatx16 acc[4];
  f16x8 hf[4][2][2];  // hidden B fragments: [unit block = k-chunk][k-step][term]
  auto mfma3 = [](const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, floatx16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);  // smallest terms first
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  };

  int p = P0;
  for (int g = g0; g < g1; ++g) {
#pragma unroll
    for (int L = 0; L < 3; ++L) {  // (unrolled: the fragment arrays are indexed by compile-time k-chunks)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[ob][i] = 0.f;
      const int nkc = L == 0 ? KC0 : 4;
#pragma unroll
      for (int kc = 0; kc < nkc; ++kc, ++p) {
        if (p + RING - 1 < NP) wait_vm_lgkm<(RING - 2) * PIECES>();
        else wait_vm_lgkm<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (p + RING - 1 < NP) issue(p + RING - 1);
        const char* base = lds + (p % RING) * PHASE;
#pragma unroll
        for (int obp = 0; obp < 2; ++obp) {
          f16x8 fa[2][2][2];  // [unit block of the pair][k-step][term]
#pragma unroll
          for (int ob = 0; ob < 2; ++ob)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const char* half = base + obp * SLAB + ob * 4096;
              const int o = slab_off(r32, 16 * t + 8 * h);
              fa[ob][t][0] = *reinterpret_cast<const f16x8*>(half + o);
              fa[ob][t][1] = *reinterpret_cast<const f16x8*>(half + 2048 + o);
            }
#pragma unroll
          for (int ob = 0; ob < 2; ++ob)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              f16x8 bh, bl;
              if (L == 0) {
                bh = xb[2 * kc + t][0];
                bl = xb[2 * kc + t][1];
              } else {
                bh = hf[kc][t][0];
                bl = hf[kc][t][1];
              }
              acc[2 * obp + ob] = mfma3(fa[ob][t][0], fa[ob][t][1], bh, bl, acc[2 * obp + ob]);
            }
        }
      }
      // ---- layer epilogue: z = acc / (s_act s_u) + b_u, ReLU ----
      const float* pl = s_par + (g * 3 + L) * 256;
      float mx = 0.f;
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) {
        const float2* pp = reinterpret_cast<const float2*>(pl) + (ob * 2 + h) * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float2 wb = pp[i];
          const float z = fmaxf(acc[ob][i] * (act_inv * wb.x) + wb.y, 0.f);
          acc[ob][i] = z;
          mx = fmaxf(mx, z);
        }
      }
      if (L < 2) {  // split into the next layer's B fragments, scaled by this hidden row's exact maximum
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const int e = (mx > 0.f && mx <= 3.4028235e38f) ? row_exp(mx) + 2 : 0;
        const float sc = ldexpf(1.f, e);
        act_inv = ldexpf(1.f, -e);
#pragma unroll
        for (int ob = 0; ob < 4; ++ob)
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            unsigned uh[4], ul[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float x0 = acc[ob][8 * st + 2 * k] * sc, x1 = acc[ob][8 * st + 2 * k + 1] * sc;
              uh[k] = sfx::pk_f16(x0, x1);
              const sfx::sfx_f16x2 hh = __builtin_bit_cast(sfx::sfx_f16x2, uh[k]);
              ul[k] = sfx::pk_f16(x0 - (float)hh.x, x1 - (float)hh.y);
            }
            hf[ob][st][0] = __builtin_bit_cast(f16x8, make_uint4(uh[0], uh[1], uh[2], uh[3]));
            hf[ob][st][1] = __builtin_bit_cast(f16x8, make_uint4(ul[0], ul[1], ul[2], ul[3]));
          }
      } else {  // output layer on the VALU (fp32), partner lanes hold the two halves of the 128 units
        const int c0 = a.ocol[g], c1 = a.ocol[g + 1];
        const float* w4 = s_par + W4_OFF;
        const float* b4 = s_par + b4_off(a.out_dim);
        for (int c = c0; c < c1; ++c) {
          const float* wr = w4 + c * HW;
          float s = 0.f;
#pragma unroll
          for (int ob = 0; ob < 4; ++ob)
#pragma unroll
            for (int i = 0; i < 16; ++i) s = fmaf(wr[32 * ob + acc_row(i, h)], acc[ob][i], s);
          s += __shfl_xor(s, 32, 64);
          if (h == 0 && pok) {
            float z = s + b4[c];
            if (c < a.n_tanh) z = tanhf(z);
            Y[(long long)prow * a.out_dim + c] = X[(long long)prow * ldx + a.res_off + c] + z;
          }
        }
      }
    }
    act_inv = in_inv;  // next head: the input row again
  }
}

// ---- packing (once per weight version) ------------------------------------------------------------------------
// row exponents of every weight row of layers 1..3 (max in [2^14, 2^15))
__global__ void heads_rowexp_kernel(int rows, int cols, const float* __restrict__ W, int* __restrict__ e_out) {
  const int row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float m = 0.f;
  for (int c = lane; c < cols; c += 64) m = fmaxf(m, fabsf(W[(long long)row * cols + c]));
  m = sfx::wave_max(m);
  if (lane == 0) e_out[row] = (m > 0.f && m <= 3.4028235e38f) ? row_exp(m) + 2 : 0;
}

// slab stream: for head g: layer 0 k-chunks 0..KP/32-1, then layers 1, 2 k-chunks 0..3; each phase = 2 slabs
// (unit-block pairs), each slab [2 blocks][2 terms][32 rows][32 positions] (swizzled, slab_off).  One thread per
// (phase, slab, block, row, position).
__global__ void heads_pack_stream_kernel(int ng, int kp, int kin, const float* __restrict__ w1, int ld1,
                                         const float* __restrict__ wm, const int* __restrict__ e1,
                                         const int* __restrict__ em, float* __restrict__ stream) {
  const int kc0 = kp / 32, pph = kc0 + 8;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)ng * pph * 2 * 2 * 32 * 32;
  if (idx >= total) return;
  const int q = (int)(idx & 31), r = (int)((idx >> 5) & 31), obl = (int)((idx >> 10) & 1), obp = (int)((idx >> 11) & 1);
  const long long ph = idx >> 12;
  const int g = (int)(ph / pph), pq = (int)(ph % pph);
  const int u = 32 * (2 * obp + obl) + r;  // unit (row of the layer's weight)
  float w;
  int e;
  if (pq < kc0) {  // layer 0: input channel 32 kc + q
    const int in = 32 * pq + q;
    w = in < kin ? w1[(long long)(g * HW + u) * ld1 + in] : 0.f;
    e = e1[g * HW + u];
  } else {
    const int L = (pq - kc0) / 4 + 1, kc = (pq - kc0) % 4;
    const int s = q >> 4, hh = (q >> 3) & 1, jj = q & 7;
    const int in = 32 * kc + 16 * s + 8 * (jj >> 2) + 4 * hh + (jj & 3);
    w = wm[(((long long)(L - 1) * ng + g) * HW + u) * HW + in];
    e = em[((L - 1) * ng + g) * HW + u];
  }
  const float x = w * ldexpf(1.f, e);
  const _Float16 hv = (_Float16)x;
  const _Float16 lv = (_Float16)(x - (float)hv);
  char* slab = reinterpret_cast<char*>(stream) + ph * PHASE + obp * SLAB + obl * 4096;
  *reinterpret_cast<_Float16*>(slab + slab_off(r, q)) = hv;
  *reinterpret_cast<_Float16*>(slab + 2048 + slab_off(r, q)) = lv;
}

__global__ void heads_pack_params_kernel(int ng, int out_dim, const float* __restrict__ b1,
                                         const float* __restrict__ bm, const int* __restrict__ e1,
                                         const int* __restrict__ em, const float* __restrict__ w4,
                                         const float* __restrict__ b4, float* __restrict__ par) {
  const int t = (int)blockIdx.x * 256 + threadIdx.x;
  if (t < ng * 3 * HW) {  // (g, L, slot) with slot = (ob * 2 + h) * 16 + i
    const int slot = t % HW, gl = t / HW, g = gl / 3, L = gl % 3;
    const int i = slot & 15, hh = (slot >> 4) & 1, ob = slot >> 5;
    const int u = 32 * ob + acc_row(i, hh);
    const int e = L == 0 ? e1[g * HW + u] : em[((L - 1) * ng + g) * HW + u];
    const float b = L == 0 ? b1[g * HW + u] : bm[((L - 1) * ng + g) * HW + u];
    par[(g * 3 + L) * 256 + 2 * slot] = ldexpf(1.f, -e);
    par[(g * 3 + L) * 256 + 2 * slot + 1] = b;
  }
  if (t < out_dim * HW) par[W4_OFF + t] = w4[t];
  if (t < out_dim) par[b4_off(out_dim) + t] = b4[t];
}

inline bool heads_ok(int ng, int kin, int out_dim) {
  return ng >= 1 && ng <= MAXH && kin >= 1 && kin <= 160 && out_dim >= 1 && out_dim <= 64;
}

}  // namespace

extern "C" {

size_t sfx_heads_stream_floats(int ng, int kin) {
  const int kp = kin <= 128 ? 128 : 160;
  return (size_t)ng * (kp / 32 + 8) * PHASE / 4;
}
size_t sfx_heads_params_floats(int out_dim) { return (size_t)b4_off(out_dim) + out_dim + 1; }

// w1 [ng*128, ld1] (first layers, concatenated; kin used columns), wm [2][ng][128][128] (layers 2, 3), b1 [ng*128],
// bm [2][ng][128], w4 [out_dim][128] (each output row's weights over its own head's 128 units), b4 [out_dim];
// ws: (ng * 128 * 3) ints of scratch
int sfx_heads_pack(int ng, int kin, int out_dim, const float* w1, int ld1, const float* b1, const float* wm,
                   const float* bm, const float* w4, const float* b4, float* stream, float* params, int* ws,
                   void* stream_) {
  SFX_REQUIRE(heads_ok(ng, kin, out_dim) && ld1 >= kin, "sfx_heads_pack: unsupported head shape");
  SFX_REQUIRE(w1 && b1 && wm && bm && w4 && b4 && stream && params && ws, "sfx_heads_pack: null buffer");
  hipStream_t st = sfx::as_stream(stream_);
  const int kp = kin <= 128 ? 128 : 160;
  int* e1 = ws;
  int* em = ws + ng * HW;
  heads_rowexp_kernel<<<sfx::ceil_div(ng * HW, 4), 256, 0, st>>>(ng * HW, ld1, w1, e1);
  heads_rowexp_kernel<<<sfx::ceil_div(2 * ng * HW, 4), 256, 0, st>>>(2 * ng * HW, HW, wm, em);
  const long long total = (long long)ng * (kp / 32 + 8) * 4096;
  heads_pack_stream_kernel<<<sfx::ceil_div(total, 256), 256, 0, st>>>(ng, kp, kin, w1, ld1, wm, e1, em, stream);
  const int pt = ng * 3 * HW > out_dim * HW ? ng * 3 * HW : out_dim * HW;
  heads_pack_params_kernel<<<sfx::ceil_div(pt, 256), 256, 0, st>>>(ng, out_dim, b1, bm, e1, em, w4, b4, params);
  return sfx::check_launch("sfx_heads_pack");
}

// Y [M, out_dim] = heads(X[:, :kin]) + X[:, res_off : res_off + out_dim], tanh on the first n_tanh columns
int sfx_heads(int M, int ng, int kin, int out_dim, const float* x, long long ldx, int res_off, int n_tanh,
              const int* ocols, const float* stream, const float* params, float* y, void* stream_) {
  SFX_REQUIRE(M >= 0 && heads_ok(ng, kin, out_dim), "sfx_heads: unsupported head shape");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(x && ocols && stream && params && y && ldx >= kin && res_off + out_dim <= ldx,
              "sfx_heads: bad arguments");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(stream) & 15) == 0 && ldx % 4 == 0 &&
                  (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (long long)M * ldx * 4 + 64 < (long long)OOB,
              "sfx_heads: alignment / size");
  HeadsArgs a;
  a.ng = ng;
  a.kin = kin;
  a.out_dim = out_dim;
  a.res_off = res_off;
  a.n_tanh = n_tanh;
  for (int g = 0; g <= MAXH; ++g) a.ocol[g] = g <= ng ? ocols[g] : out_dim;
  SFX_REQUIRE(a.ocol[0] == 0 && a.ocol[ng] == out_dim, "sfx_heads: column table");
  const int npar = (int)sfx_heads_params_floats(out_dim);
  hipStream_t st = sfx::as_stream(stream_);
  const unsigned blocks = sfx::ceil_div(M, WAVES * 32);
  // one workgroup per CU: a launch of B point blocks takes ceil(B / CUs) rounds; splitting every block's heads into S
  // groups (grid.y) makes the rounds S times shorter, so the last, partly empty round costs 1/S of one (config B:
  // 391 blocks = 1.53 rounds -> 2 at S = 1, 5 / 3 at S = 3).  Each group re-reads and re-splits its input rows and
  // stages the parameters again: S is the smallest that reaches the best rounds x (1 / S) + 7 % per extra group (the
  // measured overhead: B 235 -> 223 us at S = 3; config E's 7.63 rounds ran 0.3 % faster per step unsplit than at S = 3,
  // profiles/r06_ab_heads_split_E.txt).
  const int cus = num_cus();
  static const bool split_on = !(getenv("SFX_HEADS_SPLIT") && !strcmp(getenv("SFX_HEADS_SPLIT"), "0"));
  int S = 1;
  double best = 1e30;
  for (int s = 1; s <= (split_on ? ng : 1); ++s) {
    if (ng % s) continue;
    const double cost = (double)sfx::ceil_div((long long)blocks * s, cus) / s * (1.0 + 0.07 * (s - 1));
    if (cost < best - 1e-9) {
      best = cost;
      S = s;
    }
  }
  const int gper = ng / S;
  const dim3 grid(blocks, (unsigned)S);
  const size_t dyn = (size_t)npar * 4;
  if (kin <= 128)
    heads_kernel<128><<<grid, WAVES * 64, dyn, st>>>(M, x, ldx, stream, params, npar, a, y, gper);
  else
    heads_kernel<160><<<grid, WAVES * 64, dyn, st>>>(M, x, ldx, stream, params, npar, a, y, gper);
  return sfx::check_launch("sfx_heads");
}

}  // extern "C"
